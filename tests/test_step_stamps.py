"""tools/step_stamps.py: launch recovery and per-class anatomy from synthetic stamp records (CPU)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("step_stamps", os.path.join(ROOT, "tools", "step_stamps.py"))
step_stamps = importlib.util.module_from_spec(spec)
spec.loader.exec_module(step_stamps)


def _rec(tag, gx, gy, t0, t1, t2, t3, wave=0, bx=0):
    return [tag, gx | (gy << 32), bx, t0, t1, t2, t3, wave]


def test_launches_split_on_time_and_kind():
    ring = 1 | 5 << 8
    recs = [
        _rec(ring, 128, 2, 100, 300, 1100, 1200), _rec(ring, 128, 2, 110, 320, 1150, 1300, wave=1),
        # same kind and grid, starts after the first launch's last t3: a second launch
        _rec(ring, 128, 2, 1400, 1600, 2400, 2500),
        _rec(2 | 3 << 8, 64, 1, 2600, 2700, 2750, 2800),
    ]
    L = step_stamps.launches(recs[::-1])
    assert [len(la["recs"]) for la in L] == [2, 1, 1]
    assert L[0]["t3max"] == 1300


def test_analyse_reports_phases_in_us():
    ring = 1 | 5 << 8
    recs = [_rec(ring, 128, 2, 0, 200, 1000, 1100), _rec(ring, 128, 2, 100, 300, 1100, 1300)]
    text = step_stamps.analyse({"streams": 64, "steps": 1, "records": recs})
    row = [ln for ln in text.splitlines() if ln.startswith("| ring mode 5")][0].split("|")
    cells = [c.strip() for c in row[1:-1]]
    assert cells[1] == "128x2"
    assert float(cells[4]) == 13.0  # span: 0 -> 1300 ticks
    assert float(cells[5]) == 1.0   # start spread
    assert float(cells[6]) == 2.0   # first load
    assert float(cells[7]) == 8.0   # stream
