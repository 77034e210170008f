"""CPU: the streaming object's host logic (gsdrxStreamPlan, include/gsdr/stream.h) against a
brute-force model: over random chunk sequences every output is produced exactly once, in order, by
the first call after which its whole window [mD, mD + W) has arrived; seam outputs read only the
history plus the declared chunk head; direct outputs read only the chunk; the history kept is exactly
the samples the next output needs and is always shorter than one window."""
import numpy as np
import pytest

from gsdr_amd.stream import plan


def brute(D, W, S, m_next, M):
    S_new = S + M
    outs = []
    m = m_next
    while m * D + W <= S_new:
        outs.append(m)
        m += 1
    return outs


@pytest.mark.parametrize("D,W", [(1, 1), (1, 63), (4, 127), (4, 131), (3, 200), (8, 8), (16, 5), (5, 1)])
def test_plan_matches_brute_force(D, W):
    rng = np.random.default_rng(D * 1000 + W)
    for trial in range(40):
        S, m_next = 0, 0
        produced = []
        for call in range(30):
            M = int(rng.choice([0, 1, 2, W - 1, W, W + 1, int(rng.integers(0, 4 * W + 40))]))
            M = max(M, 0)
            n_seam, head, n_main, main_off, hist_after = plan(D, W, S, m_next, M)
            want = brute(D, W, S, m_next, M)
            assert n_seam + n_main == len(want)
            got = list(range(m_next, m_next + n_seam + n_main))
            assert got == want
            h0 = m_next * D
            h = max(S - h0, 0)
            assert h < W  # history is always shorter than one window
            for i, m in enumerate(got):
                lo, hi = m * D, m * D + W
                if i < n_seam:  # seam: window inside history [h0, S) + chunk head [S, S + head)
                    assert lo >= h0 and lo < S and hi <= S + head
                    assert head <= M
                else:  # direct: window inside the chunk
                    assert lo >= S and hi <= S + M
                    assert lo - S == main_off + (i - n_seam) * D
            if n_seam:
                assert (n_seam - 1) * D + W == h + head  # the seam buffer holds exactly what it needs
            S_new = S + M
            m_end = m_next + len(want)
            assert hist_after == max(S_new - m_end * D, 0) and hist_after < W
            produced += got
            S, m_next = S_new, m_end
        assert produced == list(range(len(produced)))
        assert produced == brute(D, W, 0, 0, S)
