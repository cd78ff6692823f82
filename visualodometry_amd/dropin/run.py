"""Run the reference's ``src/main.py`` unchanged on the MI355X back end.

    python -m visualodometry_amd.dropin.run /path/to/VisualOdometry/src/main.py --dataset kitti ...

``sys.path`` gets this drop-in directory first (its ``config`` package is the
reference's ``VOConfig`` plus the BA knobs, default off) and the reference's
``src/`` second (its ``modules`` package, which needs cv2 & co. from the
caller's environment); :func:`hooks.install` then patches the matcher and the
keyframe hook and ``main.py`` runs as ``__main__`` with the remaining argv.
"""

import runpy
import sys
from pathlib import Path


def main(argv=None) -> None:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        raise SystemExit(__doc__)
    main_py = Path(argv.pop(0)).resolve()
    src = main_py.parent
    here = Path(__file__).resolve().parent
    sys.path[:0] = [str(here), str(src)]
    from visualodometry_amd import _lib

    _lib.load()  # fail loudly without the HIP library: there is no CPU fallback
    from visualodometry_amd.dropin import hooks

    hooks.install()
    sys.argv = [str(main_py)] + argv
    runpy.run_path(str(main_py), run_name="__main__")


if __name__ == "__main__":
    main()
