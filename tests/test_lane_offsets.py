"""The evaluator kernels' lane -> (individual, rollout) -> trajectory-row offset arithmetic
(mtgp_kernels.hip lane_place / lane_setup; loff = p * R + r, rows of P * R elements; the Acrobot
mask's fit_hist rows k * P * R + loff), restated and checked on the CPU.

The round-4 illegal address (profiles/r04/v4_pytest_gpu_fault.log) came from an uncommitted
inline-asm store experiment in the EnvAcrobotMask kernel at P = 48, R = 16: there the engine widens
the lane set to 64 (one individual per wave, lanes 16..63 inactive), and an inactive lane's
offset p * R + r reaches past its row -- past the array for the last individual.  The kernels
never store from an inactive lane (every trajectory / fit_hist store sits under `active`); this
test pins the arithmetic for active lanes, and scripts/debug_store_check.py runs the GPU suite on
the bounds-checking debug build (MTGP_DEBUG_CHECKS) to show no store is ever out of its row."""
import numpy as np
import pytest

WAVE = 64


def lane_places(P, R, lanes):
    """(wave, lane) -> (active, p, r, loff) for a launch, as lane_setup computes it (identity
    schedule: the schedule only permutes which slot q holds which individual)."""
    Rp = lanes if lanes > 0 else 1 << max(R - 1, 0).bit_length()
    out = []
    if Rp <= WAVE:
        G, W = WAVE // Rp, 1
    else:
        G, W = 1, Rp // WAVE
    waves = -(-P // G) * W
    for wv in range(waves):
        for lane in range(WAVE):
            if Rp <= WAVE:
                q0, g, r = wv * G, lane // Rp, lane % Rp
            else:
                q0, part = wv // W, wv % W
                g, r = 0, part * WAVE + lane
            if q0 >= P:
                continue
            q = q0 + g
            p = q if q < P else P  # P marks a padding group
            active = r < R and q < P
            out.append((active, p, r, p * R + r))
    return out


CASES = [(48, 16, 64), (48, 16, 0), (40, 8, 0), (40, 8, 32), (9, 1, 0), (9, 33, 0), (11, 65, 0), (11, 200, 0),
         (8192, 32, 0), (1024, 16, 64), (7, 3, 64), (13, 5, 16)]


@pytest.mark.parametrize("P,R,lanes", CASES)
def test_active_lane_offsets_cover_rows_exactly(P, R, lanes):
    places = lane_places(P, R, lanes)
    act = [(p, r, loff) for a, p, r, loff in places if a]
    PR = P * R
    loffs = np.array([x[2] for x in act])
    assert len(act) == PR and loffs.min() == 0 and loffs.max() == PR - 1
    assert len(np.unique(loffs)) == PR  # every (individual, rollout) exactly once
    assert all(0 <= p < P and 0 <= r < R for p, r, _ in act)
    S = 7
    hist = np.array([k * PR + loff for k in range(S) for loff in loffs])  # fit_hist rows [S, P * R]
    assert hist.min() >= 0 and hist.max() < S * PR


def test_inactive_lanes_reach_past_the_row():
    """Why an unmasked store faults: at the round-4 fault's shape (P 48, R 16, lane set 64) the
    inactive lanes of the last wave compute offsets up to P * R + 47 past their row."""
    places = lane_places(48, 16, 64)
    worst = max(loff for a, p, r, loff in places if not a)
    assert worst == 47 * 16 + 63 and worst >= 48 * 16


def test_kernel_stores_are_guarded_by_active():
    """Every trajectory store of the kernels is issued under `active` (source check of the save
    paths): the store_row calls sit in `if (TRAJ && active ...)` blocks or the Dopri5 save rounds
    (`on` = a live lane), and the mask's fit_save runs only `if (active)`."""
    import os
    import re
    src = open(os.path.join(os.path.dirname(__file__), "..", "multitreegp_amd", "csrc", "mtgp_kernels.hip")).read()
    # the guarded blocks: every store_row call is preceded (within its block) by one of these guards
    guard = re.compile(r"if \((TRAJ && )?[^)]*\bactive\b|if \(!on\) return;")
    # (store_row: the time-major rows; traj_put_dp: the adaptive kernels' rows in either layout, ABI v20)
    pos = [m.start() for m in re.finditer(r"(store_row(<true>)?|traj_put_dp)\(A\.out\.", src)]
    assert len(pos) > 20
    for p in pos:
        window = src[max(0, p - 1200):p]
        assert guard.search(window), src[p - 200:p + 80]
    for m in re.finditer(r"env\.fit_save\(", src):
        assert "if (active)" in src[m.start() - 40:m.start()] or "if (!on) return;" in src[m.start() - 600:m.start()]
