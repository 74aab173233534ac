"""GPU parity for the Common Coin path against the committed oracle
fixtures tests/golden/coin_n{4,7,128}.npz (tests/golden/make_coin_golden.py; N = 128 is BASELINE
config 4's shape): hash_g2 of the nonces, HBX_SHARE_* status of every signature share (including
an honest share plus a cofactor-part point, which must be rejected as off-subgroup), combined
signature, master verification, parity, and the producer-side SecretKeyShare::sign.  Bit-exact."""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _load(n):
    name = n if isinstance(n, str) else f"coin_n{n}"
    return dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))


def _digest(ctx, d):
    from hbbft_amd.hbx import DIGEST_SHA3_256, DIGEST_SHA256

    ctx.set_digest(DIGEST_SHA3_256 if str(d.get("digest", "sha256")) == "sha3_256" else DIGEST_SHA256)


def _nonces(d):
    off = d["nonce_off"]
    return [d["nonce_blob"][int(off[j]):int(off[j + 1])].tobytes() for j in range(len(off) - 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("lanes", [0, 1, 2])
@pytest.mark.parametrize("n", [4, 7, 128, "coin_n4_sha3"])
def test_coin_matches_golden(hbx_ctx, n, lanes):
    """lanes: the signature-share check on one lane per check, on two (k_verify_sig_shares2), or
    the automatic choice (two below a full chip: these fixtures)."""
    d = _load(n)
    _digest(hbx_ctx, d)
    hbx_ctx.set_verify_lanes(lanes)
    assert (hbx_ctx.set_pk_shares([r.tobytes() for r in d["pk_comp"]]) == 0).all()
    h = hbx_ctx.prepare_nonces(_nonces(d))
    np.testing.assert_array_equal(h, d["h"])
    valid = hbx_ctx.verify_sig_shares(d["sigs"], d["present"])
    np.testing.assert_array_equal(valid, d["expect_valid"])
    count, nn = d["sigs"].shape[:2]
    np.testing.assert_array_equal(hbx_ctx.sig_share_status(count, nn), d["expect_share_status"])
    sig, st, ok, par = hbx_ctx.combine_signatures(d["master_pk"].tobytes(), int(d["t"]))
    np.testing.assert_array_equal(st, d["expect_status"])
    good = st == 0
    np.testing.assert_array_equal(sig[good], d["expect_sig"][good])
    np.testing.assert_array_equal(ok[good], d["expect_master_ok"][good])
    np.testing.assert_array_equal(par[good], d["expect_parity"][good])
    assert ok[good].all()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [7, 128])
def test_two_lane_coin_fallback_matches_golden(hbx_ctx, n):
    """The two-lane coin check's fallback: a pair whose compressed squarings meet g3 = 0 (forced
    here for every third sender) is sent back -- Miller loop again, final exponentiation without
    compressed runs -- and decided with the same statuses as the fixture."""
    d = _load(n)
    _digest(hbx_ctx, d)
    hbx_ctx.set_verify_lanes(2)
    assert (hbx_ctx.set_pk_shares([r.tobytes() for r in d["pk_comp"]]) == 0).all()
    hbx_ctx.prepare_nonces(_nonces(d))
    hbx_ctx.debug_force_fallback(3)
    try:
        valid = hbx_ctx.verify_sig_shares(d["sigs"], d["present"])
        assert hbx_ctx.fallback_lanes() > 0
    finally:
        hbx_ctx.debug_force_fallback(0)
    np.testing.assert_array_equal(valid, d["expect_valid"])
    count, nn = d["sigs"].shape[:2]
    np.testing.assert_array_equal(hbx_ctx.sig_share_status(count, nn), d["expect_share_status"])
    hbx_ctx.verify_sig_shares(d["sigs"], d["present"])
    assert hbx_ctx.fallback_lanes() == 0  # nothing reaches the fallback unforced


@pytest.mark.gpu
@pytest.mark.parametrize("n", [4, 128, "coin_n4_sha3"])
def test_sign_matches_honest_shares(hbx_ctx, n):
    d = _load(n)
    _digest(hbx_ctx, d)
    hbx_ctx.prepare_nonces(_nonces(d))
    sigs = hbx_ctx.sign(d["sk"])
    honest = d["expect_valid"]
    np.testing.assert_array_equal(sigs[honest], d["sigs"][honest])


@pytest.mark.gpu
def test_hash_g2_many_nonces_vs_oracle(hbx_ctx):
    """hash_g2 (threshold_crypto G2::rand from a SHA-256-seeded ChaChaRng, full cofactor) for 256
    random messages of 0..1100 bytes, through the group kernel (16-candidate residuosity test,
    cofactor clearing on 8-16 cooperating lanes), against the oracle's sequential hash_g2: the
    compressed points must be identical."""
    import random

    from oracle import bls12_381 as bls
    from oracle import threshold as tc

    rnd = random.Random(2024)
    lens = [0, 1, 32, 63, 64, 65, 128, 1100] + [rnd.randrange(0, 1100) for _ in range(248)]
    msgs = [bytes(rnd.getrandbits(8) for _ in range(n)) for n in lens]
    _digest(hbx_ctx, {})
    h = hbx_ctx.prepare_nonces(msgs)
    for j, m in enumerate(msgs):
        assert bytes(h[j]) == bls.g2_compress(tc.hash_g2(m)), f"message {j} (len {len(m)})"


@pytest.mark.gpu
def test_hash_g2_sha3_digest_vs_oracle(hbx_ctx):
    """hash_g2 under DIGEST = SHA3-256 (hbx_set_digest): 64 messages vs the oracle."""
    import random

    from hbbft_amd.hbx import DIGEST_SHA256, DIGEST_SHA3_256
    from oracle import bls12_381 as bls
    from oracle import threshold as tc

    rnd = random.Random(77)
    msgs = [bytes(rnd.getrandbits(8) for _ in range(rnd.randrange(0, 400))) for _ in range(64)]
    hbx_ctx.set_digest(DIGEST_SHA3_256)
    try:
        h = hbx_ctx.prepare_nonces(msgs)
    finally:
        hbx_ctx.set_digest(DIGEST_SHA256)
    for j, m in enumerate(msgs):
        assert bytes(h[j]) == bls.g2_compress(tc.hash_g2(m, "sha3_256")), j


@pytest.mark.gpu
def test_verify_sigs_matches_golden(hbx_ctx):
    """PublicKey::verify batches (DHB votes votes.rs:151-156, key-generation messages
    dynamic_honey_badger.rs:395-410) against tests/golden/sigs_n16.npz:
    valid, wrong message, wrong key, off-subgroup / undecodable signature and key, identity cases."""
    from hbbft_amd.hbx import DIGEST_SHA256

    d = _load("sigs_n16")
    hbx_ctx.set_digest(DIGEST_SHA256)
    off = d["msg_off"]
    msgs = [d["msg_blob"][int(off[i]):int(off[i + 1])].tobytes() for i in range(len(off) - 1)]
    st = hbx_ctx.verify_sigs(d["pk"], msgs, d["sig"])
    np.testing.assert_array_equal(st, d["expect"])
    # a batch of one and the independence from the coin state: the same verdicts item by item
    for i in (0, 6, 8, 12):
        np.testing.assert_array_equal(hbx_ctx.verify_sigs(d["pk"][i:i + 1], msgs[i:i + 1], d["sig"][i:i + 1]),
                                      d["expect"][i:i + 1])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["bivar_t2", "bivar_t5"])
def test_bivar_commitment_checks_match_golden(hbx_ctx, name):
    """SyncKeyGen: BivarCommitment::row(our_idx + 1) (sync_key_gen.rs:313)
    and handle_ack's value check commit.evaluate(x, y) == g1 * val (:449) against
    tests/golden/bivar_t{2,5}.npz: row points byte-exact, per-ack status incl. wrong values,
    non-canonical values and an undecodable commitment."""
    d = _load(name)
    t, x = int(d["t"]), int(d["x"])
    rows, st = hbx_ctx.bivar_rows(d["commits"], t, x)
    np.testing.assert_array_equal(st, d["commit_status"])
    ok = d["commit_status"] == 1
    np.testing.assert_array_equal(rows[ok], d["rows"][ok])
    out = hbx_ctx.bivar_check_acks(d["commits"], t, x, d["ack_proposer"], d["ack_y"], d["vals"])
    np.testing.assert_array_equal(out, d["expect"])
