"""GPU parity: threshold decryption path vs the committed oracle fixtures (SURVEY.md §8 rows A1,
A2, A4-A8, f1, f2) at every BASELINE config (tests/golden/make_golden.py): N = 4, 7 (every edge
case), N = 10 (config 1), N = 64 (config 2, a full epoch), N = 256 (config 3, four proposer
columns incl. a 1 MiB ciphertext).  Bit-exact: HBX_CT_* / HBX_SHARE_* statuses, validity bits,
hoisted H_j bytes, per-proposer combine status and plaintext bytes, in the three-call host API,
the fused device call and own-share mode; producer side (public keys, encrypt, decryption shares)."""
import hashlib
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
FIXTURES = ["hb_epoch_n4", "hb_epoch_n7", "hb_epoch_n10", "hb_epoch_n64", "hb_cols_n256", "hb_epoch_n7_sha3"]


def _load(name):
    return dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))


def _cts(d):
    off = d["v_off"]
    return [(d["u"][j].tobytes(), d["v_blob"][int(off[j]):int(off[j + 1])].tobytes(), d["w"][j].tobytes())
            for j in range(len(off) - 1)]


def _check_plain(d, j, pt: bytes, own=False):
    key = "expect_plain_sha_own" if own else "expect_plain_sha"
    assert hashlib.sha256(pt).digest() == d[key][j].tobytes(), f"plaintext {j}"


def _set_keys(ctx, d):
    """Era keys plus the fixture's DIGEST variant (hbx_set_digest)."""
    from hbbft_amd.hbx import DIGEST_SHA3_256, DIGEST_SHA256

    ctx.set_digest(DIGEST_SHA3_256 if str(d["digest"]) == "sha3_256" else DIGEST_SHA256)
    st = ctx.set_pk_shares([row.tobytes() for row in d["pk_comp"]])
    assert (st == 0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("name", FIXTURES)
def test_epoch_matches_golden(hbx_ctx, name):
    d = _load(name)
    _set_keys(hbx_ctx, d)
    p, n = d["shares"].shape[:2]
    ct_ok = hbx_ctx.prepare_ciphertexts(_cts(d))
    np.testing.assert_array_equal(ct_ok, d["expect_ct_valid"])
    np.testing.assert_array_equal(hbx_ctx.ct_status(p), d["expect_ct_status"])
    # H_j = hash_g1_g2(U_j, V_j) bytes for every ciphertext that decodes
    h = hbx_ctx.ct_hashes(p)
    dec = d["expect_ct_status"] != 3
    np.testing.assert_array_equal(h[dec], d["h"][dec])
    valid = hbx_ctx.verify_dec_shares(d["shares"], d["present"])
    np.testing.assert_array_equal(valid, d["expect_valid"])
    np.testing.assert_array_equal(hbx_ctx.share_status(p, n), d["expect_share_status"])
    plains, status = hbx_ctx.combine_decrypt(int(d["t"]))
    np.testing.assert_array_equal(status, d["expect_status"])
    for j, pt in enumerate(plains):
        if status[j] == 0:
            _check_plain(d, j, pt)


def _device_epoch(ctx, d, own: bool):
    import torch

    dev = torch.device("cuda", 0)
    p, n = d["shares"].shape[:2]
    off = d["v_off"].astype(np.int64)
    t_u = torch.from_numpy(np.ascontiguousarray(d["u"])).to(dev)
    t_w = torch.from_numpy(np.ascontiguousarray(d["w"])).to(dev)
    t_v = torch.from_numpy(np.ascontiguousarray(d["v_blob"]).copy() if len(d["v_blob"]) else np.zeros(1, np.uint8)).to(dev)
    t_off = torch.from_numpy(off).to(dev)
    t_sh = torch.from_numpy(np.ascontiguousarray(d["shares"])).to(dev)
    t_pr = torch.from_numpy(np.ascontiguousarray(d["present"]).astype(np.uint8)).to(dev)
    t_out = torch.zeros(max(int(off[-1]), 1), dtype=torch.uint8, device=dev)
    t_valid = torch.zeros(p * n, dtype=torch.uint8, device=dev)
    t_ct = torch.zeros(p, dtype=torch.uint8, device=dev)
    t_st = torch.zeros(p, dtype=torch.int32, device=dev)
    maxv = int(np.max(np.diff(off))) if p else 0
    # default stream: the tensors above were uploaded on torch's current stream, and the binding
    # enqueues on that same stream (no extra synchronisation needed)
    ctx.decrypt_epoch_d(t_u, t_v, t_off, t_w, p, maxv, t_sh, n, int(d["t"]), t_out, d_valid=t_valid,
                        d_ct_valid=t_ct, d_status=t_st, d_present=t_pr)
    sfx = "_own" if own else ""
    np.testing.assert_array_equal(t_ct.cpu().numpy(), d["expect_ct_status"])
    np.testing.assert_array_equal(t_valid.cpu().numpy().reshape(p, n), d["expect_share_status" + sfx])
    status = t_st.cpu().numpy()
    np.testing.assert_array_equal(status, d["expect_status" + sfx])
    out = t_out.cpu().numpy()
    for j in range(p):
        if status[j] == 0:
            _check_plain(d, j, out[off[j]:off[j + 1]].tobytes(), own)


@pytest.mark.gpu
@pytest.mark.parametrize("name", FIXTURES)
def test_fused_epoch_call_matches_golden(hbx_ctx, name):
    """hbx_decrypt_epoch_d: statuses, combine statuses and plaintexts of the fixture in one call
    (Ciphertext::verify deferred into the share-check launch)."""
    d = _load(name)
    _set_keys(hbx_ctx, d)
    _device_epoch(hbx_ctx, d, own=False)


@pytest.mark.gpu
@pytest.mark.parametrize("name", FIXTURES)
def test_own_share_mode_matches_golden(hbx_ctx, name):
    """hbx_set_own_share: node `me`'s own share replaces its input row, and that share's check is
    Ciphertext::verify.  Host API (immediate ct checks) and the fused device call."""
    d = _load(name)
    _set_keys(hbx_ctx, d)
    me = int(d["own_me"])
    p, n = d["shares"].shape[:2]
    hbx_ctx.set_own_share(me, d["own_sk"].tobytes())
    try:
        ct_ok = hbx_ctx.prepare_ciphertexts(_cts(d))
        np.testing.assert_array_equal(ct_ok, d["expect_ct_valid"])
        valid = hbx_ctx.verify_dec_shares(d["shares"], d["present"])
        np.testing.assert_array_equal(valid, d["expect_valid_own"])
        np.testing.assert_array_equal(hbx_ctx.share_status(p, n), d["expect_share_status_own"])
        plains, status = hbx_ctx.combine_decrypt(int(d["t"]))
        np.testing.assert_array_equal(status, d["expect_status_own"])
        for j, pt in enumerate(plains):
            if status[j] == 0:
                _check_plain(d, j, pt, own=True)
        _device_epoch(hbx_ctx, d, own=True)
    finally:
        hbx_ctx.set_own_share(me, None)


@pytest.mark.gpu
def test_epochs_in_flight_on_two_contexts():
    """Two epochs in flight (bench.py epochs_in_flight; HoneyBadger handles up to max_future_epochs
    at once): one context and stream each, issued back to back without synchronising in between.
    Contexts share nothing, so each epoch's statuses and plaintexts are those of the fixture."""
    import torch

    from hbbft_amd.hbx import Context

    dev = torch.device("cuda", 0)
    ds = [_load("hb_epoch_n64"), _load("hb_epoch_n7")]
    ctxs = [Context(0), Context(0)]
    try:
        runs = []
        for ctx, d in zip(ctxs, ds):
            _set_keys(ctx, d)
            p, n = d["shares"].shape[:2]
            off = d["v_off"].astype(np.int64)
            up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
            t = dict(u=up(d["u"]), w=up(d["w"]), v=up(d["v_blob"].copy() if len(d["v_blob"]) else np.zeros(1, np.uint8)),
                     off=up(off), sh=up(d["shares"]), pr=up(d["present"].astype(np.uint8)),
                     out=torch.zeros(max(int(off[-1]), 1), dtype=torch.uint8, device=dev),
                     valid=torch.zeros(p * n, dtype=torch.uint8, device=dev),
                     ct=torch.zeros(p, dtype=torch.uint8, device=dev), st=torch.zeros(p, dtype=torch.int32, device=dev))
            runs.append((ctx, d, t, p, n, off, torch.cuda.Stream(dev)))
        torch.cuda.synchronize(dev)
        for _ in range(3):  # repeated, so later epochs overlap earlier ones on the other stream
            for ctx, d, t, p, n, off, st in runs:
                ctx.decrypt_epoch_d(t["u"], t["v"], t["off"], t["w"], p, int(np.max(np.diff(off))), t["sh"], n,
                                    int(d["t"]), t["out"], d_valid=t["valid"], d_ct_valid=t["ct"], d_status=t["st"],
                                    d_present=t["pr"], stream=st.cuda_stream)
        torch.cuda.synchronize(dev)
        for ctx, d, t, p, n, off, st in runs:
            np.testing.assert_array_equal(t["ct"].cpu().numpy(), d["expect_ct_status"])
            np.testing.assert_array_equal(t["valid"].cpu().numpy().reshape(p, n), d["expect_share_status"])
            status = t["st"].cpu().numpy()
            np.testing.assert_array_equal(status, d["expect_status"])
            out = t["out"].cpu().numpy()
            for j in range(p):
                if status[j] == 0:
                    _check_plain(d, j, out[off[j]:off[j + 1]].tobytes())
    finally:
        for ctx in ctxs:
            ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["hb_epoch_n64", "hb_epoch_n7"])
def test_device_calls_then_host_calls(hbx_ctx, name):
    """_d calls on a caller's stream (not synchronised by the caller), then host calls on the
    context's own stream (every entry point orders after this context's previous work
    on any stream).  The host combine and status readouts must see the device calls' results."""
    import torch

    d = _load(name)
    _set_keys(hbx_ctx, d)
    dev = torch.device("cuda", 0)
    p, n = d["shares"].shape[:2]
    off = d["v_off"].astype(np.int64)
    up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    t_u, t_w, t_off = up(d["u"]), up(d["w"]), up(off)
    t_v = up(d["v_blob"].copy() if len(d["v_blob"]) else np.zeros(1, np.uint8))
    t_sh, t_pr = up(d["shares"]), up(d["present"].astype(np.uint8))
    torch.cuda.synchronize(dev)
    side = torch.cuda.Stream(dev)
    hbx_ctx.prepare_ciphertexts_d(t_u, t_v, t_off, t_w, p, int(np.max(np.diff(off))), stream=side.cuda_stream)
    hbx_ctx.verify_dec_shares_d(t_sh, n, p, d_present=t_pr, stream=side.cuda_stream)
    # no synchronisation here: the host calls below must order themselves after the side stream
    plains, status = hbx_ctx.combine_decrypt(int(d["t"]))
    np.testing.assert_array_equal(hbx_ctx.share_status(p, n), d["expect_share_status"])
    np.testing.assert_array_equal(hbx_ctx.ct_status(p), d["expect_ct_status"])
    np.testing.assert_array_equal(status, d["expect_status"])
    for j, pt in enumerate(plains):
        if status[j] == 0:
            _check_plain(d, j, pt)


@pytest.mark.gpu
def test_unknown_sender_status(hbx_ctx):
    """Senders >= n of hbx_set_pk_shares: HBX_SHARE_UNKNOWN_SENDER (the reference returns
    Err(UnknownSender), honey_badger.rs:64-66), never a verification."""
    d = _load("hb_epoch_n7")
    n = d["shares"].shape[1]
    _set_keys(hbx_ctx, d)
    hbx_ctx.set_pk_shares([row.tobytes() for row in d["pk_comp"][: n - 2]])
    p = d["shares"].shape[0]
    hbx_ctx.prepare_ciphertexts(_cts(d))
    hbx_ctx.verify_dec_shares(d["shares"], d["present"])
    st = hbx_ctx.share_status(p, n)
    want = d["expect_share_status"].copy()
    want[:, n - 2:] = np.where(d["present"][:, n - 2:], 5, 2)
    np.testing.assert_array_equal(st, want)


@pytest.mark.gpu
def test_combine_needs_verify_after_prepare(hbx_ctx):
    """A prepare invalidates the previous verification: combine before the next verify is an
    error (HBX_E_NO_CIPHERTEXTS), not a decryption with the old shares."""
    from hbbft_amd.hbx import HBX_E_NO_CIPHERTEXTS, HbxError

    d = _load("hb_epoch_n4")
    _set_keys(hbx_ctx, d)
    hbx_ctx.prepare_ciphertexts(_cts(d))
    hbx_ctx.verify_dec_shares(d["shares"], d["present"])
    hbx_ctx.prepare_ciphertexts(_cts(d))
    with pytest.raises(HbxError) as e:
        hbx_ctx.combine_decrypt(int(d["t"]))
    assert e.value.code == HBX_E_NO_CIPHERTEXTS


@pytest.mark.gpu
def test_key_change_clears_own_share(hbx_ctx):
    """hbx_set_pk_shares starts a new era: the own share of the old keys is dropped, so the next
    epoch runs in plain mode instead of checking ciphertexts with a stale secret."""
    d = _load("hb_epoch_n7")
    _set_keys(hbx_ctx, d)
    hbx_ctx.set_own_share(int(d["own_me"]), d["own_sk"].tobytes())
    _set_keys(hbx_ctx, d)  # new era (same keys here): own share cleared
    _device_epoch(hbx_ctx, d, own=False)


# ---- producer side ------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("name", ["hb_epoch_n7", "hb_epoch_n64", "hb_cols_n256"])
def test_public_keys_match_oracle(hbx_ctx, name):
    d = _load(name)
    np.testing.assert_array_equal(hbx_ctx.public_keys(d["sk_shares"]), d["pk_comp"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["hb_epoch_n7", "hb_epoch_n10", "hb_cols_n256", "hb_epoch_n7_sha3"])
def test_encrypt_matches_oracle(hbx_ctx, name):
    """PublicKey::encrypt with given r_j: U, V, W bytes equal the oracle's (honey_badger.rs:116)."""
    d = _load(name)
    _set_keys(hbx_ctx, d)
    off = d["enc_msg_off"]
    p = len(off) - 1
    msgs = [d["enc_msg_blob"][int(off[j]):int(off[j + 1])].tobytes() for j in range(p)]
    cts = hbx_ctx.encrypt(d["master_pk"].tobytes(), msgs, d["enc_r"])
    voff = d["v_off"]
    for j in range(p):
        if not d["enc_ok"][j]:
            continue
        u, v, w = cts[j]
        assert u == d["enc_u"][j].tobytes(), f"U {j}"
        assert w == d["enc_w"][j].tobytes(), f"W {j}"
        assert v == d["v_blob"][int(voff[j]):int(voff[j + 1])].tobytes(), f"V {j}"


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["hb_epoch_n7", "hb_epoch_n64", "hb_cols_n256"])
def test_decrypt_shares_match_oracle(hbx_ctx, name):
    """decrypt_share_no_verify: S_ji = sk_i U_j bytes equal the fixture's honest shares."""
    d = _load(name)
    keep = d["enc_ok"] & (d["expect_ct_status"] != 3)
    u = d["enc_u"][keep]
    sh = hbx_ctx.decrypt_shares(d["sk_shares"], u)
    want = d["shares"][keep]
    mask = ~d["corrupt"][keep] & d["present"][keep] & (d["expect_share_status"][keep] != 3)
    np.testing.assert_array_equal(sh[mask], want[mask])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["hb_epoch_n7", "hb_epoch_n64", "hb_cols_n256"])
def test_one_lane_combine_matches_golden(hbx_ctx, name):
    """The fixtures' launches are small, so the default path runs the quad combine (k_combine_q);
    this forces the one-lane-per-term combine (k_combine: what a full N = 256 epoch on one GPU
    uses) through the same plaintext and status expectations."""
    d = _load(name)
    _set_keys(hbx_ctx, d)
    hbx_ctx.set_combine_lanes(1)
    try:
        _device_epoch(hbx_ctx, d, own=False)
    finally:
        hbx_ctx.set_combine_lanes(0)


@pytest.mark.gpu
@pytest.mark.parametrize("lanes", [1, 2, 3, 7])
@pytest.mark.parametrize("name", ["hb_epoch_n4", "hb_epoch_n7", "hb_epoch_n10", "hb_epoch_n64", "hb_cols_n256",
                                  "hb_epoch_n7_sha3"])
def test_one_lane_checks_match_golden(hbx_ctx, name, lanes):
    """The fixtures' launches are small, so the default (auto) path above runs the six-lane
    share check (pairing3d.hpp check2_g6d); this forces the one-lane path (what a full N = 256
    epoch on one GPU uses: the Miller kernel + the seven final-exponentiation step kernels of
    fe1d.hpp), the single-kernel one-lane check (7), the two-lane kernel (pairing2d.hpp) and the
    three-lane kernel through the same expectations, plain and own-share mode."""
    d = _load(name)
    _set_keys(hbx_ctx, d)
    hbx_ctx.set_verify_lanes(lanes)
    try:
        _device_epoch(hbx_ctx, d, own=False)
        assert hbx_ctx.verify_lanes_used() == lanes
        hbx_ctx.set_own_share(int(d["own_me"]), d["own_sk"].tobytes())
        try:
            _device_epoch(hbx_ctx, d, own=True)
        finally:
            hbx_ctx.set_own_share(0, None)
    finally:
        hbx_ctx.set_verify_lanes(0)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["hb_epoch_n10", "hb_cols_n256"])
def test_one_lane_fallback_path_matches_golden(hbx_ctx, name):
    """The one-lane path's fallback (a lane whose compressed squarings meet g3 = 0 is decided again
    by the single-kernel check): forced on every third sender's lane, same statuses, plaintexts
    and own-share ciphertext verdicts."""
    d = _load(name)
    _set_keys(hbx_ctx, d)
    hbx_ctx.set_verify_lanes(1)
    hbx_ctx.debug_force_fallback(3)
    try:
        _device_epoch(hbx_ctx, d, own=False)
        assert hbx_ctx.fallback_lanes() > 0  # the forced lanes did take the fallback check
        hbx_ctx.set_own_share(int(d["own_me"]), d["own_sk"].tobytes())
        try:
            _device_epoch(hbx_ctx, d, own=True)
        finally:
            hbx_ctx.set_own_share(0, None)
    finally:
        hbx_ctx.debug_force_fallback(0)
        hbx_ctx.set_verify_lanes(0)


def degenerate_epoch():
    """Two ciphertexts at N = 4 (oracle crypto), the first built with r = m = 3(x^2 - 1) mod r: then
    W = [m] H = H' and every honest share is S_i = [m] pk_i, so both Miller pairs of a check use
    H''s lines at P and -P, f lies in Fq6 and the easy part of the final exponentiation gives 1
    (the compressed squarings would start at g3 = 0).  One share of each ciphertext is
    another sender's (invalid)."""
    from oracle import bls12_381 as bls
    from oracle import threshold as tc
    from oracle.chacha_rand04 import ChaChaRng04

    n = 4
    sks = tc.SecretKeySet.random(1, ChaChaRng04([0x68626278, 0x72656D, 5]))
    pks = sks.public_keys()
    m = 3 * (bls.BLS_X ** 2 - 1) % bls.R
    cts = [tc.encrypt(pks.public_key(), msg, r) for msg, r in ((b"r = 3(x^2 - 1)", m), (b"any other r", 0x1234567))]
    shares = np.zeros((2, n, 48), dtype=np.uint8)
    expect = np.ones((2, n), dtype=bool)
    for j, ct in enumerate(cts):
        for i in range(n):
            src = (i + 1) % n if i == 2 else i
            shares[j, i] = np.frombuffer(bls.g1_compress(tc.decrypt_share(sks.secret_key_share(src), ct)), np.uint8)
        expect[j, 2] = False
    wire = [(bls.g1_compress(u), v, bls.g2_compress(w)) for u, v, w in cts]
    pk_comp = [bls.g1_compress(pks.public_key_share(i)) for i in range(n)]
    return sks, pks, cts, wire, pk_comp, shares, expect


@pytest.mark.gpu
def test_degenerate_ciphertext_r_m(hbx_ctx):
    """A ciphertext with r = 3(x^2 - 1) (degenerate_epoch): its honest shares verify, the forged
    one does not, and no one-lane check is sent to the fallback (k_fe1<0> decides t = 1); the
    own-share lane gives Ciphertext::verify = valid.  Lanes 1 (steps), 7 (single kernel), 6, 3."""
    _, _, _, wire, pk_comp, shares, expect = degenerate_epoch()
    sks = degenerate_epoch()[0]
    assert (hbx_ctx.set_pk_shares(pk_comp) == 0).all()
    try:
        for lanes in (1, 7, 6, 3):
            hbx_ctx.set_verify_lanes(lanes)
            assert hbx_ctx.prepare_ciphertexts(wire).all()
            np.testing.assert_array_equal(hbx_ctx.verify_dec_shares(shares), expect)
            assert hbx_ctx.verify_lanes_used() == lanes
            if lanes == 1:
                assert hbx_ctx.fallback_lanes() == 0
        hbx_ctx.set_verify_lanes(1)
        hbx_ctx.set_own_share(1, sks.secret_key_share(1).to_bytes(32, "big"))
        try:
            assert hbx_ctx.prepare_ciphertexts(wire).all()
            np.testing.assert_array_equal(hbx_ctx.verify_dec_shares(shares), expect)
            assert hbx_ctx.fallback_lanes() == 0
            np.testing.assert_array_equal(hbx_ctx.ct_status(2), [1, 1])
        finally:
            hbx_ctx.set_own_share(0, None)
    finally:
        hbx_ctx.set_verify_lanes(0)
