"""Host-side key material for synthetic epochs (mirror of the reference's test key generation).

Reference: ``NetworkInfo::generate_map`` (src/messaging.rs:359-401) draws
``SecretKeySet::random(num_faulty)`` -- a random polynomial of degree f = (N-1)//3 over Fr
(src/messaging.rs:258) -- and gives node i the secret share ``poly(i + 1)`` (threshold_crypto
``SecretKeySet::secret_key_share``); the master key is ``poly(0)``.  Public keys are derived on the
GPU by ``hbx_public_keys``.  The reference seeds from ``thread_rng``; here the coefficients come
from a seeded numpy generator so every run (and every rank) builds the same keys.

Only Fr polynomial evaluation happens here (plain Python ints); no curve arithmetic.
"""
from __future__ import annotations

import numpy as np

FR_R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def num_faulty(n: int) -> int:
    """f = (N - 1) / 3 (src/messaging.rs:258)."""
    return (n - 1) // 3


def random_scalars(rng: np.random.Generator, count: int) -> list:
    """Uniform canonical Fr scalars (rejection-sampled 255-bit integers)."""
    out = []
    while len(out) < count:
        raw = rng.integers(0, 256, size=32, dtype=np.uint8).tobytes()
        v = int.from_bytes(raw, "big") & ((1 << 255) - 1)
        if v < FR_R:
            out.append(v)
    return out


def scalars_to_be32(vals) -> np.ndarray:
    return np.frombuffer(b"".join(int(v).to_bytes(32, "big") for v in vals), dtype=np.uint8).reshape(-1, 32).copy()


class SecretKeySet:
    """Polynomial of degree ``threshold`` over Fr (threshold_crypto ``SecretKeySet``)."""

    def __init__(self, coeffs):
        self.coeffs = [int(c) % FR_R for c in coeffs]

    @classmethod
    def random(cls, threshold: int, rng: np.random.Generator) -> "SecretKeySet":
        return cls(random_scalars(rng, threshold + 1))

    @property
    def threshold(self) -> int:
        return len(self.coeffs) - 1

    def evaluate(self, x: int) -> int:
        acc = 0
        for c in reversed(self.coeffs):
            acc = (acc * x + c) % FR_R
        return acc

    def secret_key_share(self, i: int) -> int:
        """Share of node index i (x = i + 1)."""
        return self.evaluate(i + 1)

    def secret_key(self) -> int:
        return self.coeffs[0]


def generate_keys(n: int, seed: int = 0x68626278_00000001):
    """Keys of an N-node network: (SecretKeySet, sk_i as uint8[n, 32] BE, master sk as uint8[1, 32])."""
    rng = np.random.default_rng(seed)
    sks = SecretKeySet.random(num_faulty(n), rng)
    shares = scalars_to_be32([sks.secret_key_share(i) for i in range(n)])
    master = scalars_to_be32([sks.secret_key()])
    return sks, shares, master
