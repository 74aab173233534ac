"""ChaCha20 RNG as ``rand = 0.4.2`` (reference ``Cargo.toml:29``) exposes it -- TEST ORACLE ONLY.

Restated from the published rand 0.4 ``ChaChaRng`` (confidence M):

* state = "expand 32-byte k" constants, 8 key words = the seed ``[u32; 8]`` verbatim, 4 counter
  words starting at 0 (words 12..15 form one 128-bit little-endian counter);
* 20 rounds (10 double rounds), output block = rounds(state) + state, emitted word 0..15 in order;
* ``next_u32`` returns the next block word; ``next_u64`` = ``(next_u32 << 32) | next_u32``
  (rand 0.4's default ``Rng::next_u64``);
* ``gen::<u8>()`` / ``gen::<bool>()`` consume one ``next_u32`` (low byte; bool = low bit).

threshold_crypto seeds it from a 32-byte digest read as 8 big-endian u32 words.
"""
from __future__ import annotations

import struct

_MASK = 0xFFFFFFFF
_CONST = (0x61707865, 0x3320646E, 0x79622D32, 0x6B206574)


def _rotl(x: int, n: int) -> int:
    return ((x << n) | (x >> (32 - n))) & _MASK


def _qr(s, a, b, c, d):
    s[a] = (s[a] + s[b]) & _MASK
    s[d] = _rotl(s[d] ^ s[a], 16)
    s[c] = (s[c] + s[d]) & _MASK
    s[b] = _rotl(s[b] ^ s[c], 12)
    s[a] = (s[a] + s[b]) & _MASK
    s[d] = _rotl(s[d] ^ s[a], 8)
    s[c] = (s[c] + s[d]) & _MASK
    s[b] = _rotl(s[b] ^ s[c], 7)


def chacha20_block(state):
    x = list(state)
    for _ in range(10):
        _qr(x, 0, 4, 8, 12)
        _qr(x, 1, 5, 9, 13)
        _qr(x, 2, 6, 10, 14)
        _qr(x, 3, 7, 11, 15)
        _qr(x, 0, 5, 10, 15)
        _qr(x, 1, 6, 11, 12)
        _qr(x, 2, 7, 8, 13)
        _qr(x, 3, 4, 9, 14)
    return [(x[i] + state[i]) & _MASK for i in range(16)]


class ChaChaRng04:
    def __init__(self, key_words):
        key_words = list(key_words)
        assert len(key_words) <= 8
        key_words += [0] * (8 - len(key_words))
        self.state = list(_CONST) + [k & _MASK for k in key_words] + [0, 0, 0, 0]
        self.buf = []
        self.idx = 16

    @classmethod
    def from_digest(cls, digest32: bytes) -> "ChaChaRng04":
        assert len(digest32) == 32
        return cls(struct.unpack(">8I", digest32))

    def _update(self):
        self.buf = chacha20_block(self.state)
        self.idx = 0
        for i in range(12, 16):
            self.state[i] = (self.state[i] + 1) & _MASK
            if self.state[i] != 0:
                break

    def next_u32(self) -> int:
        if self.idx == 16:
            self._update()
        v = self.buf[self.idx]
        self.idx += 1
        return v

    def next_u64(self) -> int:
        hi = self.next_u32()
        lo = self.next_u32()
        return (hi << 32) | lo

    def gen_u8(self) -> int:
        return self.next_u32() & 0xFF

    def gen_bool(self) -> bool:
        return (self.gen_u8() & 1) == 1

    def keystream_bytes(self, n: int) -> bytes:
        """n outputs of gen::<u8>() (one u32 word consumed per byte)."""
        return bytes(self.next_u32() & 0xFF for _ in range(n))
