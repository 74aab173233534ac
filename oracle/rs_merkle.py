"""reed-solomon-erasure 3.1.0 + merkle (afck/merkle.rs @ public-proof) + broadcast framing restated
-- TEST ORACLE ONLY (the checker, never the product).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this.
Restates, from the published algorithms, the un-vendored dependencies
behind hbbft's Broadcast (reference ``src/broadcast.rs``):

* ``reed-solomon-erasure = 3.1.0`` (reference ``Cargo.toml:31``): GF(2^8) with generating
  polynomial x^8+x^4+x^3+x^2+1 (0x11D) and generator 2; encoding matrix
  ``V * inverse(V[0..k])`` with ``V[r][c] = r^c`` (0^0 = 1); ``encode`` fills parity shards;
  ``reconstruct_shards`` uses the FIRST k present shards in index order, inverts that k x k
  sub-matrix, rebuilds missing data shards, then re-encodes missing parity shards; fewer than k
  present -> ``TooFewShardsPresent``.  ``Coding::Trivial`` when there are no parity shards
  (``broadcast.rs:596-658``).
* ``merkle`` (``Cargo.toml:27``) with ``ring::digest::SHA256`` (``Cargo.toml:32``): leaf =
  SHA-256(0x00 || value), node = SHA-256(0x01 || left || right); levels paired left to right,
  an odd trailing node promoted unchanged; ``gen_proof`` for the first equal leaf;
  ``Proof::validate`` (root, lemma chain, leaf hash of the value) and the fork's
  ``Proof::index``.
* Broadcast framing / glue (``broadcast.rs:332-404``, ``:660-707``): BE u32 length prefix,
  shard_len = ceil(len/k), zero padding, index byte prepended to every shard, glue of the first
  k leaves.

Parity status: the GF(2^8)/Vandermonde construction is fully specified by the crate's published
algorithm and self-checked (systematic, any-k-of-n round trips, the index-byte property of
SURVEY.md §0.7); hashing is SHA-256 (hashlib).  No reference binary could be run (no Rust), so
byte parity with the crates is pinned by these published definitions only.  One detail is
unpinned: whether the fork's ``validate`` re-hashes the proof value at the leaf (SURVEY App. A.6
says it does; this oracle does).
"""
from __future__ import annotations

import hashlib
import struct

import numpy as np

# ---------------------------------------------------------------------------------------------
# GF(2^8)  (rse galois_8: polynomial 0x11D, generator 2)
# ---------------------------------------------------------------------------------------------
GF_POLY = 0x11D
EXP = np.zeros(512, dtype=np.int64)
LOG = np.zeros(256, dtype=np.int64)
_x = 1
for _i in range(255):
    EXP[_i] = _x
    LOG[_x] = _i
    _x <<= 1
    if _x & 0x100:
        _x ^= GF_POLY
for _i in range(255, 512):
    EXP[_i] = EXP[_i - 255]

# full multiplication table for vectorised shard arithmetic
MUL = np.zeros((256, 256), dtype=np.uint8)
for _a in range(1, 256):
    MUL[_a, 1:] = EXP[LOG[_a] + LOG[np.arange(1, 256)]]


def gmul(a: int, b: int) -> int:
    return int(MUL[a, b])


def gexp(a: int, n: int) -> int:
    """galois_8::exp: a^n with 0^0 = 1."""
    if n == 0:
        return 1
    if a == 0:
        return 0
    return int(EXP[(int(LOG[a]) * n) % 255])


def ginv(a: int) -> int:
    if a == 0:
        raise ZeroDivisionError
    return int(EXP[255 - LOG[a]])


def mat_mul(A, B):
    out = [[0] * len(B[0]) for _ in range(len(A))]
    for i, row in enumerate(A):
        for k, a in enumerate(row):
            if a:
                for j, b in enumerate(B[k]):
                    if b:
                        out[i][j] ^= gmul(a, b)
    return out


def mat_inv(M):
    """Gauss-Jordan inverse over GF(2^8) (rse matrix.rs: swap in a lower row when the pivot is 0)."""
    n = len(M)
    A = [list(row) + [1 if i == j else 0 for j in range(n)] for i, row in enumerate(M)]
    for r in range(n):
        if A[r][r] == 0:
            for below in range(r + 1, n):
                if A[below][r]:
                    A[r], A[below] = A[below], A[r]
                    break
            else:
                raise ValueError("singular matrix")
        inv = ginv(A[r][r])
        A[r] = [gmul(v, inv) for v in A[r]]
        for other in range(n):
            if other != r and A[other][r]:
                f = A[other][r]
                A[other] = [v ^ gmul(f, w) for v, w in zip(A[other], A[r])]
    return [row[n:] for row in A]


def vandermonde(rows: int, cols: int):
    return [[gexp(r, c) for c in range(cols)] for r in range(rows)]


class TooFewShardsPresent(Exception):
    pass


def code_rows(rows: np.ndarray, inputs: np.ndarray) -> np.ndarray:
    """out[r] = XOR_c rows[r, c] * inputs[c] (vectorised over bytes)."""
    out = np.zeros((rows.shape[0], inputs.shape[1]), dtype=np.uint8)
    for r in range(rows.shape[0]):
        acc = np.zeros(inputs.shape[1], dtype=np.uint8)
        for c in range(rows.shape[1]):
            if rows[r, c]:
                acc ^= MUL[rows[r, c]][inputs[c]]
        out[r] = acc
    return out


class ReedSolomon:
    """reed_solomon_erasure::ReedSolomon (3.1.0): k data + m parity shards, k + m <= 256."""

    def __init__(self, data_shards: int, parity_shards: int):
        if data_shards <= 0 or parity_shards <= 0 or data_shards + parity_shards > 256:
            raise ValueError("invalid shard counts")
        self.k, self.m = data_shards, parity_shards
        v = vandermonde(self.k + self.m, self.k)
        self.matrix = mat_mul(v, mat_inv(v[: self.k]))
        self.parity_rows = np.array(self.matrix[self.k:], dtype=np.uint8)

    def encode(self, shards: np.ndarray) -> np.ndarray:
        """shards: uint8[k + m, L]; returns a copy with the parity rows filled."""
        out = np.array(shards, dtype=np.uint8, copy=True)
        out[self.k:] = code_rows(self.parity_rows, out[: self.k])
        return out

    def reconstruct(self, shards):
        """shards: list of k + m (bytes-like or None) -> list of bytes (all present)."""
        n = self.k + self.m
        present = [i for i in range(n) if shards[i] is not None]
        if len(present) == n:
            return [bytes(s) for s in shards]
        if len(present) < self.k:
            raise TooFewShardsPresent()
        sub = present[: self.k]
        sub_shards = np.stack([np.frombuffer(bytes(shards[i]), dtype=np.uint8) for i in sub])
        decode = np.array(mat_inv([self.matrix[i] for i in sub]), dtype=np.uint8)
        out = [None if s is None else np.frombuffer(bytes(s), dtype=np.uint8) for s in shards]
        missing_data = [i for i in range(self.k) if out[i] is None]
        if missing_data:
            rebuilt = code_rows(decode[missing_data], sub_shards)
            for r, i in enumerate(missing_data):
                out[i] = rebuilt[r]
        missing_parity = [i for i in range(self.k, n) if out[i] is None]
        if missing_parity:
            data = np.stack(out[: self.k])
            rebuilt = code_rows(self.parity_rows[[i - self.k for i in missing_parity]], data)
            for r, i in enumerate(missing_parity):
                out[i] = rebuilt[r]
        return [bytes(o) for o in out]


# ---------------------------------------------------------------------------------------------
# Merkle tree (merkle.rs with ring SHA-256)
# ---------------------------------------------------------------------------------------------
# Two tree digests (include/hbx.h HBX_MERKLE_*):
#   "sha256": merkle (afck fork) + ring SHA-256 -- leaf H(0x00 || v), node H(0x01 || l || r);
#   "sha3":   later hbbft's own src/broadcast/merkle.rs (tiny-keccak) -- leaf SHA3-256(v), node
#             SHA3-256(l || r); same level structure (pairs left to right, odd node promoted).
#             Restated from the published later hbbft source as remembered: parity unpinned.
def hash_leaf(value: bytes, variant: str = "sha256") -> bytes:
    if variant == "sha3":
        return hashlib.sha3_256(bytes(value)).digest()
    return hashlib.sha256(b"\x00" + bytes(value)).digest()


def hash_nodes(left: bytes, right: bytes, variant: str = "sha256") -> bytes:
    if variant == "sha3":
        return hashlib.sha3_256(left + right).digest()
    return hashlib.sha256(b"\x01" + left + right).digest()


class MerkleTree:
    """MerkleTree::from_vec: levels paired left to right, odd trailing node promoted."""

    def __init__(self, values, variant: str = "sha256"):
        self.variant = variant
        self.values = [bytes(v) for v in values]
        if not self.values:
            self.levels = [[hashlib.sha256(b"").digest()]]
            return
        level = [hash_leaf(v, variant) for v in self.values]
        self.levels = [level]
        while len(level) > 1:
            nxt = [hash_nodes(level[i], level[i + 1], variant) for i in range(0, len(level) - 1, 2)]
            if len(level) % 2:
                nxt.append(level[-1])
            self.levels.append(nxt)
            level = nxt

    def root_hash(self) -> bytes:
        return self.levels[-1][0]

    def gen_proof(self, value: bytes):
        """Proof for the FIRST leaf equal to `value` (None if absent): {root_hash, lemma, value};
        lemma = [(node_hash, sibling)] from the root down, sibling = ('L'|'R', hash) of the child
        on the path (merkle.rs Positioned), the last entry (leaf hash, None)."""
        try:
            idx = self.values.index(bytes(value))
        except ValueError:
            return None
        up = []  # (hash of the node on the path at this level, sibling) from the leaf upward
        pos = idx
        for lvl in range(len(self.levels) - 1):
            level = self.levels[lvl]
            if pos % 2 == 0 and pos == len(level) - 1:  # promoted: no node at this level
                pos //= 2
                continue
            sib = ("R", level[pos + 1]) if pos % 2 == 0 else ("L", level[pos - 1])
            up.append((level[pos], sib))
            pos //= 2
        lemma = []
        cur = self.root_hash()
        for child_hash, sib in reversed(up):
            lemma.append((cur, sib))
            cur = child_hash
        lemma.append((cur, None))
        return {"root_hash": self.root_hash(), "lemma": lemma, "value": bytes(value)}


def proof_validate(proof, root_hash: bytes, variant: str = "sha256") -> bool:
    """merkle.rs Proof::validate."""
    lemma = proof["lemma"]
    if proof["root_hash"] != root_hash or lemma[0][0] != root_hash:
        return False
    for k, (node_hash, sib) in enumerate(lemma):
        if k == len(lemma) - 1:
            return sib is None and hash_leaf(proof["value"], variant) == node_hash
        if sib is None:
            return False
        sub_hash = lemma[k + 1][0]
        combined = hash_nodes(sib[1], sub_hash, variant) if sib[0] == "L" else hash_nodes(sub_hash, sib[1], variant)
        if combined != node_hash:
            return False
    return False


def proof_index(proof, count: int) -> int:
    """Fork-only Proof::index(count): the leaf position the Left/Right path selects in the
    promote-odd tree of `count` leaves (the left subtree of a node over c leaves holds
    2^(ceil(log2 c) - 1) of them)."""
    idx, c = 0, count
    for _node_hash, sib in proof["lemma"][:-1]:
        left = 1 << ((c - 1).bit_length() - 1) if c > 1 else 1
        if sib[0] == "R":      # the path goes left
            c = left
        else:                  # the path goes right
            idx += left
            c -= left
    return idx


def validate_broadcast_proof(proof, node_index: int, n: int, variant: str = "sha256") -> bool:
    """Broadcast::validate_proof (broadcast.rs:555-575)."""
    return (proof_validate(proof, proof["root_hash"], variant) and len(proof["value"]) > 0
            and node_index == proof["value"][0] and proof_index(proof, n) == proof["value"][0])


# ---------------------------------------------------------------------------------------------
# Broadcast framing (broadcast.rs:332-404, :660-707)
# ---------------------------------------------------------------------------------------------
def num_faulty(n: int) -> int:
    return (n - 1) // 3


def coding_counts(n: int):
    """(data, parity) = (N - 2f, 2f) (broadcast.rs:310-311)."""
    f = num_faulty(n)
    return n - 2 * f, 2 * f


def frame_shards(value: bytes, n: int) -> np.ndarray:
    """BE u32 length || value, zero-padded to n * shard_len, as uint8[n, shard_len] (data rows
    filled, parity rows zero: broadcast.rs:341-353)."""
    k, _ = coding_counts(n)
    framed = struct.pack(">I", len(value)) + bytes(value)
    shard_len = -(-len(framed) // k)
    buf = np.zeros((n, shard_len), dtype=np.uint8)
    buf.reshape(-1)[: len(framed)] = np.frombuffer(framed, dtype=np.uint8)
    return buf


def send_shards(value: bytes, n: int, variant: str = "sha256"):
    """Frame, RS-encode, index-prefix: returns (shards uint8[n, L], leaves, tree)."""
    k, m = coding_counts(n)
    buf = frame_shards(value, n)
    if m > 0:
        buf = ReedSolomon(k, m).encode(buf)
    leaves = [bytes([i & 0xFF]) + buf[i].tobytes() for i in range(n)]
    return buf, leaves, MerkleTree(leaves, variant)


def glue_shards(leaves, k: int):
    data = b"".join(bytes(l)[1:] for l in leaves[:k])
    if len(data) < 4:
        return None
    ln = struct.unpack(">I", data[:4])[0]
    return data[4:4 + ln]


def decode_from_shards(leaf_values, n: int, root_hash: bytes, variant: str = "sha256"):
    """broadcast.rs:660-692: reconstruct (index byte included), rebuild the tree, compare the root,
    glue.  leaf_values: list of n (bytes or None).  Returns the value or None."""
    k, m = coding_counts(n)
    if m > 0:
        try:
            leaves = ReedSolomon(k, m).reconstruct(leaf_values)
        except TooFewShardsPresent:
            return None
    else:
        if any(v is None for v in leaf_values):
            return None
        leaves = [bytes(v) for v in leaf_values]
    if MerkleTree(leaves, variant).root_hash() != root_hash:
        return None
    return glue_shards(leaves, k)
