"""CPU tests of the measurement tools the round-5 findings rest on
(tools/slam_trace.py): a synthetic event trace in slam_rate's format, with
one slow submission, is summarised per pass as DESIGN.md §6 quotes it."""
import os
import subprocess
import sys

from conftest import ROOT


def test_slam_trace_summary_names_the_slow_submission(tmp_path):
    ev = [(0.0000, 1, 0), (0.0001, 2, 0), (0.0002, 3, 1), (0.0002, 4, 1), (0.0003, 12, 1),
          (0.0003, 12, 2), (0.0004, 12, 3), (0.0004, 12, 4), (0.0005, 12, 5), (0.0005, 5, 0),
          (0.0006, 3, 8), (0.0006, 4, 8), (0.0007, 12, 1), (0.0007, 12, 2), (0.0090, 12, 3),
          (0.0091, 12, 4), (0.0092, 12, 5), (0.0092, 5, 0), (0.0093, 6, 2), (0.0095, 7, 1)]
    p = tmp_path / "events.txt"
    p.write_text("# pass 0 100.000000000 100.010000000\n" +
                 "".join(f"{t + 100.0:.9f} {k} {a}\n" for t, k, a in ev))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "slam_trace.py"), str(p)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    out = r.stdout
    assert "pass 0:" in out and "launches 2" in out
    assert "slow submit of 8 frames" in out and "step 3 +8.400" in out
    assert "longest call submit 8.600 ms" in out
