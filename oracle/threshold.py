"""threshold_crypto restatement (hash-to-G2, threshold encryption and signatures) -- TEST ORACLE.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use it.
It restates the un-vendored, unpinned dependency ``threshold_crypto`` (reference
``Cargo.toml:35``) at the call sites hbbft's hot path uses:

* ``hash_g2`` / ``hash_g1_g2`` / ``hash_bytes``          (App. A.3)
* ``PublicKey::encrypt``, ``Ciphertext::verify``          (honey_badger.rs:116, :371)
* ``SecretKeyShare::decrypt_share_no_verify``             (honey_badger.rs:403)
* ``PublicKeyShare::verify_decryption_share``             (honey_badger.rs:229)
* ``PublicKeySet::decrypt`` (= interpolate + hash_bytes)  (honey_badger.rs:340)
* ``SecretKeyShare::sign``, ``PublicKeyShare::verify``    (common_coin.rs:142, :151)
* ``PublicKeySet::combine_signatures``, ``PublicKey::verify``, ``Signature::parity``
                                                          (common_coin.rs:190, :196, :173)
* ``Nonce::new``                                          (agreement/mod.rs:155-165)

Parity status: the verification bits and the Lagrange-combined points are canonical (they do not
depend on any unpinned detail).  Bytes that pass through the hash-to-G2 / keystream construction
(W, H, signature shares, decrypted plaintexts, parity bits) follow SURVEY.md App. A.3 with the
DIGEST = SHA-256 default; the true threshold_crypto revision is not available here, so those
bytes are "parity unpinned" against the reference (self-consistent, documented in DESIGN.md).
"""
from __future__ import annotations

import hashlib

from . import bls12_381 as bls
from .chacha_rand04 import ChaChaRng04

DIGESTS = {
    "sha256": lambda m: hashlib.sha256(m).digest(),
    "sha3_256": lambda m: hashlib.sha3_256(m).digest(),
}
DEFAULT_DIGEST = "sha256"


def digest(msg: bytes, variant: str = DEFAULT_DIGEST) -> bytes:
    return DIGESTS[variant](bytes(msg))


# ---------------------------------------------------------------------------------------------
# Rand impls of pairing 0.14 (raw Montgomery repr filled from next_u64, masked, rejection-sampled)
# ---------------------------------------------------------------------------------------------
def fq_rand(rng: ChaChaRng04) -> int:
    while True:
        limbs = [rng.next_u64() for _ in range(6)]
        limbs[5] &= 0xFFFFFFFFFFFFFFFF >> 3  # REPR_SHAVE_BITS = 384 - 381
        v = sum(l << (64 * i) for i, l in enumerate(limbs))
        if v < bls.P:
            return bls.fq_from_mont_repr(v)


def fr_rand(rng: ChaChaRng04) -> int:
    while True:
        limbs = [rng.next_u64() for _ in range(4)]
        limbs[3] &= 0xFFFFFFFFFFFFFFFF >> 1  # REPR_SHAVE_BITS = 256 - 255
        v = sum(l << (64 * i) for i, l in enumerate(limbs))
        if v < bls.R:
            return bls.fr_from_mont_repr(v)


def fq2_rand(rng: ChaChaRng04):
    c0 = fq_rand(rng)
    c1 = fq_rand(rng)
    return (c0, c1)


def g2_rand(rng: ChaChaRng04):
    """pairing 0.14 ``impl Rand for G2``: x <- Fq2::rand, greatest <- bool, lift, clear the
    cofactor with the full h2 (``scale_by_cofactor``), retry on failure or identity."""
    while True:
        x = fq2_rand(rng)
        greatest = rng.gen_bool()
        rhs = bls.f2_add(bls.f2_mul(bls.f2_sqr(x), x), bls.B2)
        y = bls.f2_sqrt(rhs)
        if y is None:
            continue
        negy = bls.f2_neg(y)
        # pairing: y if (y < negy) ^ greatest else negy
        y_lt = bls.f2_lex_gt(negy, y)
        yy = y if (y_lt ^ greatest) else negy
        p = bls.g2_mul((x, yy), bls.H2)
        if p is not None:
            return p


# ---------------------------------------------------------------------------------------------
# threshold_crypto hashes
# ---------------------------------------------------------------------------------------------
def hash_g2(msg: bytes, variant: str = DEFAULT_DIGEST):
    return g2_rand(ChaChaRng04.from_digest(digest(msg, variant)))


def hash_g1_g2(g1pt, msg: bytes, variant: str = DEFAULT_DIGEST):
    m = digest(msg, variant) if len(msg) > 64 else bytes(msg)
    return hash_g2(m + bls.g1_compress(g1pt), variant)


def hash_bytes(g1pt, n: int, variant: str = DEFAULT_DIGEST) -> bytes:
    rng = ChaChaRng04.from_digest(digest(bls.g1_compress(g1pt), variant))
    return rng.keystream_bytes(n)


def xor_bytes(a: bytes, b: bytes) -> bytes:
    return bytes(x ^ y for x, y in zip(a, b))


# ---------------------------------------------------------------------------------------------
# Keys (SecretKeySet = polynomial of degree t over Fr; index i maps to x = i + 1)
# ---------------------------------------------------------------------------------------------
class SecretKeySet:
    def __init__(self, coeffs):
        self.coeffs = list(coeffs)

    @classmethod
    def random(cls, threshold: int, rng: ChaChaRng04) -> "SecretKeySet":
        return cls([fr_rand(rng) for _ in range(threshold + 1)])

    @property
    def threshold(self) -> int:
        return len(self.coeffs) - 1

    def evaluate(self, x: int) -> int:
        acc = 0
        for c in reversed(self.coeffs):
            acc = (acc * x + c) % bls.R
        return acc

    def secret_key_share(self, i: int) -> int:
        return self.evaluate(i + 1)

    def secret_key(self) -> int:
        return self.coeffs[0] % bls.R

    def public_keys(self) -> "PublicKeySet":
        return PublicKeySet([bls.g1_mul(bls.G1_GEN, c) for c in self.coeffs])


class PublicKeySet:
    """Commitment = coefficients * g1.  ``public_key_share(i)`` = commit.evaluate(i + 1)
    (reference messaging.rs:251-254)."""

    def __init__(self, commit):
        self.commit = list(commit)

    @property
    def threshold(self) -> int:
        return len(self.commit) - 1

    def public_key(self):
        return self.commit[0]

    def public_key_share(self, i: int):
        x = i + 1
        acc = None
        for c in reversed(self.commit):
            acc = bls.g1_add(bls.g1_mul(acc, x) if acc is not None else None, c)
        return acc

    def to_bytes(self) -> bytes:
        """invocation_id = master public key bytes (messaging.rs:342-344)."""
        return bls.g1_compress(self.public_key())


# ---------------------------------------------------------------------------------------------
# Threshold encryption
# ---------------------------------------------------------------------------------------------
def encrypt(pk, msg: bytes, r: int, variant: str = DEFAULT_DIGEST):
    u = bls.g1_mul(bls.G1_GEN, r)
    g = bls.g1_mul(pk, r)
    v = xor_bytes(hash_bytes(g, len(msg), variant), msg)
    w = bls.g2_mul(hash_g1_g2(u, v, variant), r)
    return (u, v, w)


def ciphertext_verify(ct, variant: str = DEFAULT_DIGEST, hash_pt=None) -> bool:
    """e(g1, W) == e(U, H(U, V))  (honey_badger.rs:371)."""
    u, v, w = ct
    h = hash_pt if hash_pt is not None else hash_g1_g2(u, v, variant)
    return bls.pairing_product_is_one([(bls.G1_GEN, w), (bls.g1_neg(u), h)])


def decrypt_share(sk_i: int, ct):
    """S_i = sk_i * U (honey_badger.rs:403)."""
    return bls.g1_mul(ct[0], sk_i)


def verify_decryption_share(pk_i, share, ct, variant: str = DEFAULT_DIGEST, hash_pt=None) -> bool:
    """e(S_i, H(U, V)) == e(pk_i, W)  (honey_badger.rs:229).  ``hash_pt`` lets a caller hoist
    H(U, V) per ciphertext; the answer is identical."""
    u, v, w = ct
    h = hash_pt if hash_pt is not None else hash_g1_g2(u, v, variant)
    return bls.pairing_product_is_one([(share, h), (bls.g1_neg(pk_i), w)])


class NotEnoughShares(Exception):
    pass


class DuplicateEntry(Exception):
    pass


def lagrange_coeffs_at_zero(indices):
    """lambda_i(0) = prod_{j != i} x_j / (x_j - x_i), x = index + 1, over Fr."""
    xs = [i + 1 for i in indices]
    out = []
    for xi in xs:
        num, den = 1, 1
        for xj in xs:
            if xj == xi:
                continue
            num = num * xj % bls.R
            den = den * (xj - xi) % bls.R
        out.append(num * pow(den, -1, bls.R) % bls.R)
    return out


def interpolate(t: int, items, add, mul):
    """threshold_crypto ``interpolate``: take the FIRST t items, error on too few or a repeated
    index, return sum lambda_i * sample_i."""
    samples = list(items)[:t]
    if len(samples) < t:
        raise NotEnoughShares()
    idx = [i for i, _ in samples]
    if len(set(idx)) != len(idx):
        raise DuplicateEntry()
    lam = lagrange_coeffs_at_zero(idx)
    acc = None
    for l, (_, pt) in zip(lam, samples):
        acc = add(acc, mul(pt, l))
    return acc


def decrypt(pk_set: PublicKeySet, shares, ct, variant: str = DEFAULT_DIGEST) -> bytes:
    """PublicKeySet::decrypt (honey_badger.rs:340): shares is an iterable of (index, S_i) in
    index order; uses the first t = threshold + 1."""
    g = interpolate(pk_set.threshold + 1, shares, bls.g1_add, bls.g1_mul)
    return xor_bytes(hash_bytes(g, len(ct[1]), variant), ct[1])


# ---------------------------------------------------------------------------------------------
# Threshold signatures (Common Coin)
# ---------------------------------------------------------------------------------------------
def sign(sk: int, msg: bytes, variant: str = DEFAULT_DIGEST, hash_pt=None):
    h = hash_pt if hash_pt is not None else hash_g2(msg, variant)
    return bls.g2_mul(h, sk)


def verify_sig(pk, sig, msg: bytes, variant: str = DEFAULT_DIGEST, hash_pt=None) -> bool:
    """e(pk, H(m)) == e(g1, sig)  (common_coin.rs:151, :196)."""
    h = hash_pt if hash_pt is not None else hash_g2(msg, variant)
    return bls.pairing_product_is_one([(pk, h), (bls.g1_neg(bls.G1_GEN), sig)])


def combine_signatures(pk_set: PublicKeySet, shares):
    return interpolate(pk_set.threshold + 1, shares, bls.g2_add, bls.g2_mul)


def parity(sig) -> bool:
    """Signature::parity (common_coin.rs:173): XOR-fold of the 192-byte uncompressed encoding,
    then popcount parity."""
    x = 0
    for b in bls.g2_uncompress_bytes(sig):
        x ^= b
    return bin(x).count("1") % 2 == 1


def nonce_bytes(invocation_id: bytes, session_id: int, proposer_id: int, agreement_epoch: int) -> bytes:
    """agreement/mod.rs:155-165: format!("Nonce for Honey Badger {:?}@{}:{}:{}",
    invocation_id, session_id, agreement_epoch, proposer_id) with Vec<u8> Debug formatting."""
    dbg = "[" + ", ".join(str(b) for b in invocation_id) + "]"
    return f"Nonce for Honey Badger {dbg}@{session_id}:{agreement_epoch}:{proposer_id}".encode()
