"""tools/xgmi_stamps.py: the reading of a timed-out exchange launch from its per-workgroup stamps
(starvation vs a flag that was raised but not seen)."""
import importlib.util
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
spec = importlib.util.spec_from_file_location("xgmi_stamps", ROOT / "tools" / "xgmi_stamps.py")
xs = importlib.util.module_from_spec(spec)
spec.loader.exec_module(xs)

T = 5 * 10 ** 8  # 5 s in 100 MHz ticks


def _ranks(sender_start, sender_flag1):
    # rank 0 block 0 waited on rank 1 block 3's flag1 for step 7 and timed out
    r0 = {"rank": 0, "nblk": 4, "timeout_s": 5.0,
          "rows": [[0, 7, 1000, 1100, 1000 + T + 50, 1000 + T + 90, 3, 1 * 4 + 3 + 1],
                   [1, 7, 1000, 1100, 1200, 1300, 0, 0]]}
    r1 = {"rank": 1, "nblk": 4, "timeout_s": 5.0,
          "rows": [[3, 7, sender_start, sender_flag1, sender_flag1 + 10, sender_flag1 + 20, 0, 0],
                   [0, 6, 500, 600, 700, 800, 0, 0]]}
    return {0: r0, 1: r1}


def test_starvation_reading():
    res = xs.analyse(_ranks(1000 + T + 100, 1000 + T + 200))
    assert [f["step"] for f in res["failures"]] == [7]
    w = res["failures"][0]["waits"][0]
    assert w["missing_sender"] == [1, 3] and w["reading"].startswith("starvation")


def test_protocol_reading():
    w = xs.analyse(_ranks(1500, 1600))["failures"][0]["waits"][0]
    assert w["reading"].startswith("protocol")


def test_no_failure_no_reading():
    r = _ranks(1500, 1600)
    r[0]["rows"][0][6] = r[0]["rows"][0][7] = 0
    assert xs.analyse(r)["failures"] == []
