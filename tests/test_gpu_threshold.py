"""GPU parity: threshold decryption path vs the committed oracle fixtures (SURVEY.md §8 rows
A1, A2, A4, A5).  Bit-exact: validity bits, ciphertext bits, per-proposer status, plaintext bytes."""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _load(n):
    return dict(np.load(os.path.join(GOLDEN, f"hb_epoch_n{n}.npz"), allow_pickle=False))


def _cts(d):
    off = d["v_off"]
    return [(d["u"][j].tobytes(), d["v_blob"][int(off[j]):int(off[j + 1])].tobytes(), d["w"][j].tobytes())
            for j in range(len(off) - 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [4, 7])
def test_epoch_matches_golden(hbx_ctx, n):
    d = _load(n)
    st = hbx_ctx.set_pk_shares([row.tobytes() for row in d["pk_comp"]])
    assert (st == 0).all()
    ct_ok = hbx_ctx.prepare_ciphertexts(_cts(d))
    np.testing.assert_array_equal(ct_ok, d["expect_ct_valid"])
    valid = hbx_ctx.verify_dec_shares(d["shares"], d["present"])
    np.testing.assert_array_equal(valid, d["expect_valid"])
    plains, status = hbx_ctx.combine_decrypt(int(d["t"]))
    np.testing.assert_array_equal(status, d["expect_status"])
    off = d["v_off"]
    for j, pt in enumerate(plains):
        if status[j] == 0:
            assert pt == d["expect_plain_blob"][int(off[j]):int(off[j + 1])].tobytes()
