"""tools/timeline.py's parser on synthetic timing buffers (CPU): a stamp a wave never writes (0)
must drop the wave from every phase that uses it, never produce a difference against 0."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import timeline  # noqa: E402


def _row(hw, rt0, rt1, stamps):
    r = np.zeros(16, np.int64)
    r[0], r[1], r[2] = hw, rt0, rt1
    for k, v in stamps.items():
        r[3 + k] = v
    return r


def test_small_kernel_rows_with_missing_stamps():
    base = 10_000_000
    rows = []
    # two env waves (stamps 0-5, 12), on two SIMDs of XCD 0
    for w in range(2):
        s = {0: base, 1: base + 1900, 2: base + 9600, 3: base + 14900, 4: base + 16000, 12: base + 18800,
             5: base + 19700}
        rows.append(_row((0 << 32) | (w << 4), 1000, 1000 + 19700 // 24, s))
    # three helper waves: only wave 2's writes 6 and 8; none writes 1, 2, 3
    for w in range(1, 4):
        s = {0: base, 10: base + 3000, 11: base + 9000, 9: base + 12000, 4: base + 16000, 12: base + 18800,
             5: base + 19700}
        if w == 2:
            s.update({6: base + 16100, 8: base + 18500})
        rows.append(_row((1 << 32) | (w << 4), 1002, 1002 + 19700 // 24, s))
    # a wave of a launch that never ran it (all zero): must be ignored
    rows.append(np.zeros(16, np.int64))
    res = timeline.analyze(np.stack(rows), small=True)
    assert res["negative"] == 0
    ph = res["phases"]
    assert ph["env: physics"]["waves"] == 2 and ph["env: physics"]["mean"] == 7700
    assert ph["env: obs/history/stores"]["mean"] == 5300
    assert ph["env: obs row write-out"]["mean"] == 2800
    assert ph["helper: speculative reset"]["waves"] == 3 and ph["helper: speculative reset"]["mean"] == 3000
    assert ph["helper wave 2: gyro + rows + stores"]["waves"] == 1
    assert ph["helper wave 2: gyro + rows + stores"]["mean"] == 2400
    # no env phase is computed from helper waves and vice versa
    assert ph["env: wave lifetime"]["waves"] == 2 and ph["helper: wave lifetime"]["waves"] == 3
    for p in ph.values():
        assert 0 <= p["mean"] < 1e6 and p["max"] < 1e6
    assert res["simds_used"] == 5
    # the two env waves sit on two different SIMDs
    assert res["env_waves_per_simd_hist"] == {1: 2}


def test_large_kernel_rows_and_out_of_order_stamps_are_counted():
    base = 5_000_000
    rows = [_row(0, 100, 200, {0: base, 1: base + 10, 2: base + 50, 3: base + 80, 4: base + 90, 5: base + 120}),
            # a non-resetting wave: no role stamps 6-8, no stamp 12
            _row(1 << 4, 100, 200, {0: base, 1: base + 20, 2: base + 60, 3: base + 70, 4: base + 95, 5: base + 130}),
            # a role wave
            _row(2 << 4, 100, 200, {0: base, 1: base + 20, 2: base + 60, 3: base + 70, 4: base + 95, 6: base + 100,
                                     7: base + 110, 8: base + 125, 12: base + 126, 5: base + 140})]
    res = timeline.analyze(np.stack(rows), small=False)
    assert res["negative"] == 0
    assert res["phases"]["physics"]["waves"] == 3
    assert res["phases"]["reset role: pose"]["waves"] == 1 and res["phases"]["reset role: pose"]["mean"] == 10
    bad = np.stack(rows).copy()
    bad[0, 3 + 2] = base - 5          # stamp 2 before stamp 1: reported, not averaged in
    res2 = timeline.analyze(bad, small=False)
    assert res2["negative"] >= 1
    assert res2["phases"]["physics"]["waves"] == 2
    assert "negative phase durations: " in timeline.report(res2)
