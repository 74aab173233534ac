"""Pins the CPU oracle (oracle/) to known answers before it is trusted as the checker.

Anchors: the BLS12-381 generator encodings, group orders and
cofactors, pairing bilinearity / non-degeneracy, the RFC 7539 ChaCha20 keystream (rand 0.4
ChaChaRng with the all-zero seed is that keystream), SHA-256 from hashlib, the Nonce format of
src/agreement/mod.rs:155-165, and threshold round trips with the reference's own semantics
(first t shares by index, x = index + 1; NotEnoughShares / DuplicateEntry)."""
import pytest

from oracle import bls12_381 as bls
from oracle import threshold as tc
from oracle.chacha_rand04 import ChaChaRng04

G1_GEN_COMP = bytes.fromhex(
    "97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb")
G2_GEN_COMP = bytes.fromhex(
    "93e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e"
    "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8")


def test_constants():
    x = bls.BLS_X
    assert bls.R == x**4 - x**2 + 1
    assert bls.P == ((x + 1) ** 2 * (x**4 - x**2 + 1)) // 3 - x  # p = (z-1)^2 r / 3 + z with z = -x
    assert bls.H2.bit_length() == 507 and bin(bls.H2).count("1") == 247


def test_generator_encodings():
    assert bls.g1_compress(bls.G1_GEN) == G1_GEN_COMP
    assert bls.g2_compress(bls.G2_GEN) == G2_GEN_COMP
    assert bls.g1_decompress(G1_GEN_COMP) == bls.G1_GEN
    assert bls.g2_decompress(G2_GEN_COMP) == bls.G2_GEN
    assert bls.g1_on_curve(bls.G1_GEN) and bls.g2_on_curve(bls.G2_GEN)
    assert bls.g1_mul(bls.G1_GEN, bls.R) is None and bls.g2_mul(bls.G2_GEN, bls.R) is None
    inf = bytes([0xC0]) + bytes(47)
    assert bls.g1_compress(None) == inf and bls.g1_decompress(inf) is None


def test_bad_encodings_rejected():
    with pytest.raises(ValueError):
        bls.g1_decompress(bytes([0x9F]) + b"\xff" * 47)  # x >= p
    with pytest.raises(ValueError):
        bls.g1_decompress(bytes([G1_GEN_COMP[0] & 0x7F]) + G1_GEN_COMP[1:])  # compression flag missing


def test_pairing_bilinear_and_nondegenerate():
    a, b = 0x1234567, 0x89ABCDEF
    e = bls.pairing(bls.G1_GEN, bls.G2_GEN)
    assert e != bls.F12_ONE
    assert bls.f12_pow(e, bls.R) == bls.F12_ONE
    lhs = bls.pairing(bls.g1_mul(bls.G1_GEN, a), bls.g2_mul(bls.G2_GEN, b))
    assert lhs == bls.f12_pow(e, a * b)
    assert bls.pairing_product_is_one([(bls.g1_mul(bls.G1_GEN, a), bls.G2_GEN),
                                       (bls.g1_neg(bls.G1_GEN), bls.g2_mul(bls.G2_GEN, a))])


def test_chacha20_rfc7539_keystream():
    rng = ChaChaRng04([0] * 8)
    words = [rng.next_u32() for _ in range(16)]
    assert words == [0xADE0B876, 0x903DF1A0, 0xE56A5D40, 0x28BD8653, 0xB819D2BD, 0x1AED8DA0, 0xCCEF36A8,
                     0xC70D778B, 0x7C5941DA, 0x8D485751, 0x3FE02477, 0x374AD8B8, 0xF4B8436A, 0x1CA11815,
                     0x69B687C3, 0x8665EEB2]
    rng = ChaChaRng04([0] * 8)
    assert rng.next_u64() == (0xADE0B876 << 32) | 0x903DF1A0


def test_nonce_format():
    # src/agreement/mod.rs:161-164, invocation_id as Vec<u8> Debug
    assert tc.nonce_bytes(bytes([167, 3]), 1, 5, 2) == b"Nonce for Honey Badger [167, 3]@1:2:5"


def test_hash_g2_lands_in_g2():
    h = tc.hash_g2(b"hbbft")
    assert bls.g2_on_curve(h) and bls.g2_mul(h, bls.R) is None
    assert tc.hash_g2(b"hbbft") == h and tc.hash_g2(b"hbbfu") != h


def test_threshold_decrypt_roundtrip_and_errors():
    rng = ChaChaRng04([0x68626278, 9])
    sks = tc.SecretKeySet.random(1, rng)  # t = 2
    pks = sks.public_keys()
    msg = b"contribution of proposer 0"
    ct = tc.encrypt(pks.public_key(), msg, tc.fr_rand(rng))
    assert tc.ciphertext_verify(ct)
    shares = [(i, tc.decrypt_share(sks.secret_key_share(i), ct)) for i in range(4)]
    assert tc.verify_decryption_share(pks.public_key_share(2), shares[2][1], ct)
    assert not tc.verify_decryption_share(pks.public_key_share(1), shares[2][1], ct)
    assert tc.decrypt(pks, shares[1:3], ct) == msg
    assert tc.decrypt(pks, [shares[3], shares[0]], ct) == msg
    with pytest.raises(tc.NotEnoughShares):
        tc.decrypt(pks, shares[:1], ct)
    with pytest.raises(tc.DuplicateEntry):
        tc.decrypt(pks, [shares[1], shares[1]], ct)


def test_threshold_sign_combine_parity():
    rng = ChaChaRng04([0x68626278, 10])
    sks = tc.SecretKeySet.random(1, rng)
    pks = sks.public_keys()
    nonce = tc.nonce_bytes(tc.PublicKeySet.to_bytes(pks), 0, 0, 2)
    h = tc.hash_g2(nonce)
    sig_shares = [(i, tc.sign(sks.secret_key_share(i), nonce, hash_pt=h)) for i in range(4)]
    assert tc.verify_sig(pks.public_key_share(1), sig_shares[1][1], nonce, hash_pt=h)
    s1 = tc.combine_signatures(pks, sig_shares[:2])
    s2 = tc.combine_signatures(pks, sig_shares[2:])
    assert s1 == s2 == tc.sign(sks.secret_key(), nonce, hash_pt=h)
    assert tc.verify_sig(pks.public_key(), s1, nonce, hash_pt=h)
    assert tc.parity(s1) in (True, False)
