"""Host key generation (hbbft_amd/netinfo.py) against the oracle's Lagrange interpolation:
any t = f + 1 secret-key shares interpolate to the master key (the property the reference's
tests/sync_key_gen.rs:61-80 checks through combine_signatures)."""
from hbbft_amd import netinfo
from oracle import bls12_381 as bls
from oracle import threshold as tc


def test_generate_keys_threshold_property():
    n = 10
    sks, shares, master = netinfo.generate_keys(n, seed=7)
    f = netinfo.num_faulty(n)
    assert f == 3 and sks.threshold == f
    vals = [int.from_bytes(shares[i].tobytes(), "big") for i in range(n)]
    assert all(v < bls.R for v in vals)
    for subset in ([0, 1, 2, 3], [9, 4, 2, 7]):
        lam = tc.lagrange_coeffs_at_zero(subset)
        rec = sum(l * vals[i] for l, i in zip(lam, subset)) % bls.R
        assert rec == int.from_bytes(master[0].tobytes(), "big")


def test_generate_keys_deterministic():
    a = netinfo.generate_keys(4)[1]
    b = netinfo.generate_keys(4)[1]
    assert (a == b).all()
