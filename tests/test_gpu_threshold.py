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


@pytest.mark.gpu
@pytest.mark.parametrize("n", [4, 7])
def test_fused_epoch_call_matches_golden(hbx_ctx, n):
    """hbx_decrypt_epoch_d (Ciphertext::verify on the second stream beside the speculative
    combine) gives the fixture's bits, statuses and plaintexts, invalid ciphertext included."""
    import torch

    d = _load(n)
    assert (hbx_ctx.set_pk_shares([row.tobytes() for row in d["pk_comp"]]) == 0).all()
    dev = torch.device("cuda", 0)
    p = len(d["v_off"]) - 1
    nn = d["shares"].shape[1]
    off = d["v_off"].astype(np.int64)
    t_u = torch.from_numpy(np.ascontiguousarray(d["u"])).to(dev)
    t_w = torch.from_numpy(np.ascontiguousarray(d["w"])).to(dev)
    t_v = torch.from_numpy(np.ascontiguousarray(d["v_blob"]).astype(np.uint8).copy() if len(d["v_blob"]) else np.zeros(1, np.uint8)).to(dev)
    t_off = torch.from_numpy(off).to(dev)
    t_sh = torch.from_numpy(np.ascontiguousarray(d["shares"])).to(dev)
    t_pr = torch.from_numpy(np.ascontiguousarray(d["present"]).astype(np.uint8)).to(dev)
    t_out = torch.zeros(max(int(off[-1]), 1), dtype=torch.uint8, device=dev)
    t_valid = torch.zeros(p * nn, dtype=torch.uint8, device=dev)
    t_ct = torch.zeros(p, dtype=torch.uint8, device=dev)
    t_st = torch.zeros(p, dtype=torch.int32, device=dev)
    maxv = int(np.max(np.diff(off))) if p else 0
    hbx_ctx.decrypt_epoch_d(t_u, t_v, t_off, t_w, p, maxv, t_sh, nn, int(d["t"]), t_out, d_valid=t_valid,
                            d_ct_valid=t_ct, d_status=t_st, d_present=t_pr)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(t_ct.cpu().numpy(), d["expect_ct_valid"])
    np.testing.assert_array_equal(t_valid.cpu().numpy().reshape(p, nn), d["expect_valid"].reshape(p, nn))
    status = t_st.cpu().numpy()
    np.testing.assert_array_equal(status, d["expect_status"])
    out = t_out.cpu().numpy()
    for j in range(p):
        if status[j] == 0:
            assert out[off[j]:off[j + 1]].tobytes() == d["expect_plain_blob"][int(off[j]):int(off[j + 1])].tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [4, 7])
def test_own_share_mode_matches_golden(hbx_ctx, n):
    """hbx_set_own_share: node `me`'s own share replaces its input row, and that share's check is
    Ciphertext::verify (no separate ciphertext checks).  The fixture's own-mode expectations come
    from the oracle (tests/golden/make_golden.py): the invalid ciphertext is still caught, and the
    starved proposer gains our honest share."""
    d = _load(n)
    assert (hbx_ctx.set_pk_shares([row.tobytes() for row in d["pk_comp"]]) == 0).all()
    me = int(d["own_me"])
    hbx_ctx.set_own_share(me, d["own_sk"].tobytes())
    try:
        ct_ok = hbx_ctx.prepare_ciphertexts(_cts(d))  # immediate Ciphertext::verify (wide path)
        np.testing.assert_array_equal(ct_ok, d["expect_ct_valid"])
        valid = hbx_ctx.verify_dec_shares(d["shares"], d["present"])
        np.testing.assert_array_equal(valid, d["expect_valid_own"])
        plains, status = hbx_ctx.combine_decrypt(int(d["t"]))
        np.testing.assert_array_equal(status, d["expect_status_own"])
        off = d["v_off"]
        for j, pt in enumerate(plains):
            if status[j] == 0:
                assert pt == d["expect_plain_blob_own"][int(off[j]):int(off[j + 1])].tobytes()
        # deferred ciphertext checks: the own share's lane decides ct validity
        import torch

        dev = torch.device("cuda", 0)
        p = len(off) - 1
        t_u = torch.from_numpy(np.ascontiguousarray(d["u"])).to(dev)
        t_w = torch.from_numpy(np.ascontiguousarray(d["w"])).to(dev)
        t_v = torch.from_numpy(np.ascontiguousarray(d["v_blob"]).copy()).to(dev)
        t_off = torch.from_numpy(off.astype(np.int64)).to(dev)
        t_sh = torch.from_numpy(np.ascontiguousarray(d["shares"])).to(dev)
        t_pr = torch.from_numpy(np.ascontiguousarray(d["present"]).astype(np.uint8)).to(dev)
        t_out = torch.zeros(max(int(off[-1]), 1), dtype=torch.uint8, device=dev)
        t_valid = torch.zeros(p * n, dtype=torch.uint8, device=dev)
        t_ct = torch.zeros(p, dtype=torch.uint8, device=dev)
        t_st = torch.zeros(p, dtype=torch.int32, device=dev)
        hbx_ctx.decrypt_epoch_d(t_u, t_v, t_off, t_w, p, int(np.max(np.diff(off))), t_sh, n, int(d["t"]), t_out,
                                d_valid=t_valid, d_ct_valid=t_ct, d_status=t_st, d_present=t_pr)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(t_ct.cpu().numpy(), d["expect_ct_valid"])
        np.testing.assert_array_equal(t_valid.cpu().numpy().reshape(p, n), d["expect_valid_own"])
        np.testing.assert_array_equal(t_st.cpu().numpy(), d["expect_status_own"])
    finally:
        hbx_ctx.set_own_share(me, None)
