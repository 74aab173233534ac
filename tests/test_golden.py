"""The committed golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py) agree
with the oracle: hoisted hashes, ciphertext validity, a sample of share validities, status and
plaintexts.  Full recomputation is done by make_golden.py; this re-checks a bounded sample."""
import os

import numpy as np
import pytest

from oracle import bls12_381 as bls
from oracle import threshold as tc

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _load(n):
    return dict(np.load(os.path.join(GOLDEN, f"hb_epoch_n{n}.npz"), allow_pickle=False))


@pytest.mark.parametrize("n", [4, 7, 10])
def test_fixture_shape(n):
    d = _load(n)
    p = len(d["v_off"]) - 1
    assert d["shares"].shape == (p, n, 48) and d["expect_valid"].shape == (p, n)
    assert int(d["t"]) == (n - 1) // 3 + 1
    assert str(d["digest"]) == "sha256"
    # edge cases present: ShareDecryptionFailed, a valid ct, every share status but UNKNOWN_SENDER
    assert d["expect_ct_status"][0] == 0 and (d["expect_ct_status"] == 1).any()
    assert set(np.unique(d["expect_share_status"]).tolist()) == {0, 1, 2, 3, 4}
    assert d["expect_status"][0] == -7
    assert (d["expect_valid"] == (d["expect_share_status"] == 1)).all()


@pytest.mark.parametrize("name", ["hb_epoch_n64", "hb_cols_n256"])
def test_big_fixture_shape(name):
    d = dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))
    n = int(d["n"])
    p = len(d["v_off"]) - 1
    assert d["shares"].shape == (p, n, 48)
    assert (d["expect_ct_status"] == 1).all() and (d["expect_status"] == 0).all()
    # validity == not corrupted (FaultyShareAdversary positions), verified by the oracle at generation
    assert ((d["expect_share_status"] == 1) == ~d["corrupt"]).all()
    assert d["corrupt"].any()


@pytest.mark.parametrize("n", [4])
def test_fixture_against_oracle(n):
    d = _load(n)
    off = d["v_off"]
    p = len(off) - 1
    pks = [bls.g1_decompress(r.tobytes()) for r in d["pk_comp"]]
    for j in range(p):
        u = bls.g1_decompress(d["u"][j].tobytes())
        v = d["v_blob"][int(off[j]):int(off[j + 1])].tobytes()
        w = bls.g2_decompress(d["w"][j].tobytes())
        h = tc.hash_g1_g2(u, v)
        assert bls.g2_compress(h) == d["h"][j].tobytes()
        assert tc.ciphertext_verify((u, v, w), hash_pt=h) == bool(d["expect_ct_valid"][j])
    # every share of every valid proposer: status == the oracle's decode + verification
    for j in range(p):
        if d["expect_ct_status"][j] != 1:
            assert set(d["expect_share_status"][j][d["present"][j]].tolist()) <= {4}
            continue
        u = bls.g1_decompress(d["u"][j].tobytes())
        v = d["v_blob"][int(off[j]):int(off[j + 1])].tobytes()
        w = bls.g2_decompress(d["w"][j].tobytes())
        h = bls.g2_decompress(d["h"][j].tobytes())
        for i in range(n):
            st = int(d["expect_share_status"][j, i])
            if not d["present"][j, i]:
                assert st == 2
                continue
            try:
                s = bls.g1_decompress(d["shares"][j, i].tobytes())
            except ValueError:
                assert st == 3
                continue
            ok = tc.verify_decryption_share(pks[i], s, (u, v, w), hash_pt=h)
            assert st == (1 if ok else 0), (j, i)


@pytest.mark.parametrize("n", [4])
def test_coin_fixture_against_oracle(n):
    d = dict(np.load(os.path.join(GOLDEN, f"coin_n{n}.npz"), allow_pickle=False))
    off = d["nonce_off"]
    nonces = [d["nonce_blob"][int(off[j]):int(off[j + 1])].tobytes() for j in range(len(off) - 1)]
    for j, nonce in enumerate(nonces):
        assert nonce.startswith(b"Nonce for Honey Badger [")
        assert bls.g2_compress(tc.hash_g2(nonce)) == d["h"][j].tobytes()
    # combined signature of instance 0 verifies under the master key and has the stored parity
    sig = bls.g2_decompress(d["expect_sig"][0].tobytes())
    h0 = bls.g2_decompress(d["h"][0].tobytes())
    assert tc.verify_sig(bls.g1_decompress(d["master_pk"].tobytes()), sig, nonces[0], hash_pt=h0)
    assert tc.parity(sig) == bool(d["expect_parity"][0])


def test_c5_fixture_against_oracle():
    """tests/golden/c5_broadcast.npz (BASELINE config C5) is what oracle/rs_merkle.py gives for
    the seeded 1 MiB proposal: shard digests, both Merkle roots, the proof lemmas."""
    import hashlib

    from oracle import rs_merkle as rm

    g = np.load(os.path.join(GOLDEN, "c5_broadcast.npz"))
    n, plen = int(g["n"]), int(g["plen"])
    value = np.random.default_rng(int(g["seed"])).integers(0, 256, size=plen, dtype=np.uint8).tobytes()
    assert hashlib.sha256(value).digest() == g["payload_sha"].tobytes()
    shards, leaves, tree = rm.send_shards(value, n)
    assert shards.shape == (n, int(g["shard_len"]))
    for i in range(n):
        assert hashlib.sha256(shards[i].tobytes()).digest() == g["shard_sha"][i].tobytes()
    assert tree.root_hash() == g["root_sha256"].tobytes()
    assert rm.MerkleTree(leaves, "sha3").root_hash() == g["root_sha3"].tobytes()
    for j, leaf in enumerate(g["proof_leaves"]):
        p = tree.gen_proof(leaves[int(leaf)])
        assert len(p["lemma"]) - 1 == int(g["proof_depth"][j])
        for lv, (h, _sib) in enumerate(p["lemma"]):
            assert h == g["proof_nodes"][j, lv].tobytes()


def test_sig_fixture_against_oracle():
    """tests/golden/sigs_n16.npz (PublicKey::verify items, make_sig_golden.py): every decodable
    item's verdict and hash_g2 point recomputed by the oracle; every undecodable item rejected by
    the oracle's into_affine restatement."""
    d = dict(np.load(os.path.join(GOLDEN, "sigs_n16.npz"), allow_pickle=False))
    off = d["msg_off"]
    for i in range(int(d["count"])):
        msg = d["msg_blob"][int(off[i]):int(off[i + 1])].tobytes()
        if i % 4 == 0:
            assert bls.g2_compress(tc.hash_g2(msg)) == d["h"][i].tobytes()
        try:
            pk = bls.g1_decompress(d["pk"][i].tobytes())
            sig = bls.g2_decompress(d["sig"][i].tobytes())
        except ValueError:
            assert d["expect"][i] == 3
            continue
        if pk is None or sig is None:
            assert d["expect"][i] == (1 if pk is None and sig is None else 0)
            continue
        if i in (0, 6, 7, 14):
            assert tc.verify_sig(pk, sig, msg) == (d["expect"][i] == 1)


@pytest.mark.parametrize("name", ["bivar_t2", "bivar_t5"])
def test_bivar_fixture_against_oracle(name):
    """tests/golden/bivar_t*.npz (make_bivar_golden.py): rows re-derived from the committed
    commitment points, and a sample of acks re-evaluated (oracle/bivar.py)."""
    from oracle import bivar

    d = dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))
    t, x = int(d["t"]), int(d["x"])
    for q in range(int(d["p"])):
        if d["commit_status"][q] != 1:
            with pytest.raises(ValueError):
                [bls.g1_decompress(c.tobytes()) for c in d["commits"][q]]
            continue
        commit = [bls.g1_decompress(c.tobytes()) for c in d["commits"][q]]
        assert [bls.g1_compress(r) for r in bivar.row(commit, t, x)] == [r.tobytes() for r in d["rows"][q]]
        for k in np.nonzero(d["ack_proposer"] == q)[0][::4]:
            val = int.from_bytes(d["vals"][k].tobytes(), "big")
            if val >= bls.R:
                assert d["expect"][k] == 3
                continue
            ok = bivar.evaluate(commit, t, x, int(d["ack_y"][k])) == bls.g1_mul(bls.G1_GEN, val)
            assert ok == (d["expect"][k] == 1)
