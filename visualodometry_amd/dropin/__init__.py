"""Drop-in replacements for the reference's ``src/config`` and ``src/modules`` packages.

Put this directory (``visualodometry_amd/dropin``) ahead of the reference's
``src/`` on ``sys.path`` -- or copy ``config/`` and ``modules/`` over it -- and
``src/main.py`` runs unchanged with matching and BA on the MI355X back end
(INTEGRATION.md).
"""
