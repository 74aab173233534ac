"""The reconstruct set-up's reduced system (broadcast.hpp k_rs_setup_reconstruct, round 6) against
the oracle's full inverse (oracle/rs_merkle.py ReedSolomon.reconstruct, reed-solomon-erasure 3.1.0):
for the first k present shards the sub-matrix is [[I, 0], [E_p, E_m]] (present data shards first,
then the first nmd present parity shards; columns present data | missing data), so the rows of its
inverse for the missing data shards are [E_m^-1 E_p | E_m^-1].  The kernel inverts only the
nmd x nmd block E_m; this checks, in plain Python on the host, that its coefficients are exactly
the rows of the full k x k inverse the oracle takes -- for patterns with no, some and all data
shards missing.  (The GPU outputs themselves: tests/test_gpu_broadcast.py.)"""
import random

import pytest

from oracle import rs_merkle as rm


def reduced_rows(rs, present):
    k = rs.k
    sub = [i for i in range(rs.k + rs.m) if present[i]][:k]
    missing_data = [i for i in range(k) if not present[i]]
    nmd, npd = len(missing_data), k - len(missing_data)
    assert sub[:npd] == [i for i in range(k) if present[i]]
    par = sub[npd:]
    if nmd == 0:
        return sub, missing_data, []
    e_m = [[rs.matrix[p][d] for d in missing_data] for p in par]
    e_inv = rm.mat_inv(e_m)
    rows = []
    for o in range(nmd):
        row = []
        for c in range(k):
            if c >= npd:
                row.append(e_inv[o][c - npd])
            else:
                v = 0
                for r in range(nmd):
                    v ^= rm.gmul(e_inv[o][r], rs.matrix[par[r]][sub[c]])
                row.append(v)
        rows.append(row)
    return sub, missing_data, rows


@pytest.mark.parametrize("k,m", [(2, 2), (3, 4), (5, 8), (10, 14), (44, 84)])
def test_reduced_rows_equal_full_inverse(k, m):
    rs = rm.ReedSolomon(k, m)
    n = k + m
    rnd = random.Random(k * 131 + m)
    patterns = [[True] * (n - m) + [False] * m,                      # parity only (the bench's pattern)
                [False] * min(k, m) + [True] * (n - min(k, m))]       # the first data shards
    for _ in range(6):
        miss = set(rnd.sample(range(n), rnd.randint(1, m)))
        patterns.append([i not in miss for i in range(n)])
    for present in patterns:
        sub, missing_data, rows = reduced_rows(rs, present)
        full = rm.mat_inv([rs.matrix[i] for i in sub])
        assert rows == [full[d] for d in missing_data]
