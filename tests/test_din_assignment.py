"""CPU: the index arithmetic of din_forward_kernel's balanced assignment (csrc/din_fused.hip, NIT == 1:
per 1,024-sample universe, round 6) restated in Python — for every batch size the launch grid of
ceil(B / 16) workgroups covers every rank of every universe exactly once, each workgroup's live-row
count equals its live waves, and no workgroup reaches past its universe.  The ranking itself (a
counting sort by tile class) is a permutation inside a universe, so rank coverage is sample coverage;
the GPU tests pin the outputs bit for bit against contiguous blocks (test_gpu_din_plan.py)."""
import pytest

ROWS = 16       # kMlpRows: samples per workgroup
THREADS = 1024  # kMlpThreads: samples per universe (one length load per thread)


def deal(B):
    """(workgroup, wave) -> (universe, rank) for the launch of ceil(B / 16) workgroups, as the kernel
    computes it: j = g / 64, u0 = 1024 j, UB = min(1024, B - u0), UG = ceil(UB / 16), local index
    g - 64 j, rank ugl + UG * rho for the wave of snake position rho, live when rank < UB."""
    grid = (B + ROWS - 1) // ROWS
    seen = {}
    rows_of = {}
    for g in range(grid):
        j = g // (THREADS // ROWS)
        u0 = j * THREADS
        UB = min(THREADS, B - u0)
        UG = (UB + ROWS - 1) // ROWS
        ugl = g - j * (THREADS // ROWS)
        assert 0 <= ugl < UG, (B, g)  # no workgroup past its universe's share of the grid
        rows = min(ROWS, (UB - ugl + UG - 1) // UG)
        live = 0
        for w in range(ROWS):
            rho = (w & ~3) | ((3 - (w & 3)) if (w >> 2) & 1 else (w & 3))
            p = ugl + UG * rho
            if p < UB:
                live += 1
                key = (j, p)
                assert key not in seen, (B, g, w, key)
                seen[key] = (g, w)
        rows_of[g] = (rows, live)
    return seen, rows_of


@pytest.mark.parametrize("B", [17, 63, 64, 1000, 1023, 1024, 1025, 1040, 2047, 4096, 4097, 5000, 8192, 10000,
                               33 * 1024 + 5, 65536])
def test_universe_deal_covers_every_sample_once(B):
    seen, rows_of = deal(B)
    n_uni = (B + THREADS - 1) // THREADS
    for j in range(n_uni):
        UB = min(THREADS, B - j * THREADS)
        assert sorted(p for (jj, p) in seen if jj == j) == list(range(UB)), (B, j)
    assert len(seen) == B
    for g, (rows, live) in rows_of.items():
        assert rows == live, (B, g, rows, live)  # the live-row count the kernel uses is its live waves


def test_snake_order_is_a_permutation_of_the_waves():
    rhos = [(w & ~3) | ((3 - (w & 3)) if (w >> 2) & 1 else (w & 3)) for w in range(ROWS)]
    assert sorted(rhos) == list(range(ROWS))
    # ranks 0..3 on SIMDs 0..3, ranks 4..7 on SIMDs 3..0 (wave w runs on SIMD w % 4)
    assert [rhos.index(r) % 4 for r in range(8)] == [0, 1, 2, 3, 3, 2, 1, 0]
