"""Static check of the fused K2 + K3 launch's hand-off (csrc/ba_band.hip): the solver reads the
reduced system its reducers wrote in the same launch without an acquire fence, which is valid
only while EVERY load of those bytes is an sc1 load (SysLoads) issued after that wave's own
poll of the column's counter (MI355X_MICROARCH.md, hand-off table row 1).  Any other read of
A.sys must be on a path the fused launch never takes, and is marked so; an unmarked plain read
(a later edit adding one would read stale columns without an error) fails here."""
import re
from pathlib import Path

SRC = Path(__file__).resolve().parents[1] / "visualodometry_amd" / "csrc" / "ba_band.hip"


def test_every_plain_sys_read_is_marked_off_the_fused_path():
    unmarked = []
    for no, line in enumerate(SRC.read_text().splitlines(), 1):
        code = line.split("//")[0]
        if not re.search(r"\bA\.sys\b", code):
            continue
        if re.search(r"st_sc1\(A\.sys", code) or "SysLoads sysl(A.sys" in code:
            continue  # the reducers' write-through stores; the sc1 load view
        if "plain-sys-read: " not in line:
            unmarked.append((no, line.strip()))
    assert not unmarked, f"plain reads of A.sys without a not-fused marker: {unmarked}"


def test_fused_prologue_polls_before_its_loads():
    """In the fused prologue a wave issues a column's loads only in the round its own poll found
    the column's counter full (issue(u) guarded by the ballot's ready bit)."""
    text = SRC.read_text()
    i = text.index("const uint64_t nowb = __builtin_amdgcn_ballot_w64(now);")
    block = text[i:i + 300]
    for u in range(3):
        assert f"if (nowb & {1 << u}u) issue({u});" in block
    # a prologue column with a counter is issued nowhere else (the early issue is for columns
    # without one: the bottom separator, which the fused launch's reducers never write)
    assert text.count("issue(u);") == 1 and "!((waiting >> u) & 1u)) issue(u);" in text
