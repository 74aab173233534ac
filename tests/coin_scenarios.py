"""Message logs for the Common Coin replay tests.

``coin_scenario`` builds one node's receive log for a round of coin instances with the paths of
``src/common_coin.rs`` placed on purpose:
  * shares arriving before the node's own input (held, no output until ``had_input``, :170);
  * an invalid share (a valid share of another nonce) before the threshold: a fault, no
    ``try_output`` (:151-155);
  * an undecodable share (serde rejects it: no reaction) and an unknown sender
    (``Err(UnknownSender)``, :158), incl. an undecodable message from an unknown sender;
  * a duplicate sender (invalid, then valid: the BTreeMap keeps the valid one);
  * shares after termination, valid and invalid: ignored, no fault (:105-110);
  * an instance that never gets this node's input (holds shares, never outputs);
  * an instance whose threshold is crossed by our own share at input time.
``OracleCoinEngine`` is a CPU stand-in for ``hbbft_amd.common_coin.GpuCoinEngine`` on the oracle's
crypto (tests only).
"""
from __future__ import annotations

import random

import numpy as np

from oracle import bls12_381 as bls
from oracle import threshold as tc
from oracle.chacha_rand04 import ChaChaRng04

SHARE_INVALID, SHARE_VALID, SHARE_ABSENT, SHARE_UNDECODABLE = 0, 1, 2, 3


def keys(n: int, seed: int):
    f = (n - 1) // 3
    sks = tc.SecretKeySet.random(f, ChaChaRng04([0x68626278, 0x636F696E, seed]))
    return sks, sks.public_keys()


def nonces(count: int, seed: int):
    inv = bytes(range(seed % 7, seed % 7 + 5))
    return [tc.nonce_bytes(inv, s, p, 2) for s in range(2) for p in range(count // 2 + count % 2)][:count]


def coin_scenario(n: int, me, count: int, seed: int, variant: str = tc.DEFAULT_DIGEST):
    """(nonces, sks, pks, events) for node ``me`` (None: an observer)."""
    assert count >= 4 and n >= 4
    rng = random.Random(seed)
    f = (n - 1) // 3
    sks, pks = keys(n, seed)
    ns = nonces(count, seed)
    hs = [tc.hash_g2(x, variant) for x in ns]

    def share(i, inst):
        return bls.g2_compress(tc.sign(sks.secret_key_share(i), ns[inst], variant, hash_pt=hs[inst]))

    def foreign(i, inst):  # a valid share of another nonce: verifies false here
        return share(i, (inst + 1) % count)

    others = [i for i in range(n) if i != me]
    per_inst = []
    for inst in range(count):
        ev = []
        senders = others[:]
        rng.shuffle(senders)
        if inst == 0:
            # f + 1 shares before our input, then the input: our input triggers (observer: too)
            for i in senders[: f + 1]:
                ev.append(("share", i, inst, share(i, inst)))
            ev.append(("input", inst))
            ev.append(("share", senders[f + 1], inst, foreign(senders[f + 1], inst)))  # after termination
            ev.append(("share", senders[-1], inst, share(senders[-1], inst)))
        elif inst == 1:
            # input first; an invalid share and an undecodable one, duplicates, unknown senders
            ev.append(("input", inst))
            bad = senders[0]
            ev.append(("share", bad, inst, foreign(bad, inst)))
            ev.append(("share", senders[1], inst, bytes([0xE0]) + bytes(95)))  # not a point
            ev.append(("share", n + 2, inst, share(senders[2], inst)))  # unknown sender
            ev.append(("share", n + 5, inst, bytes(96)))  # unknown sender, undecodable
            ev.append(("share", bad, inst, share(bad, inst)))  # the same sender, now valid
            for i in senders[1 : f + 2]:
                ev.append(("share", i, inst, share(i, inst)))
            ev.append(("share", senders[-1], inst, b"\x00" * 96))  # after termination
        elif inst == 2:
            # never gets our input: all shares held, no output
            for i in senders:
                ev.append(("share", i, inst, share(i, inst)))
        else:
            # random interleaving of input, valid and a few invalid shares
            msgs = [("share", i, inst, share(i, inst) if rng.random() > 0.25 else foreign(i, inst)) for i in senders]
            pos = rng.randrange(len(msgs) + 1)
            msgs.insert(pos, ("input", inst))
            ev.extend(msgs)
        per_inst.append(ev)
    events = []
    cursors = [0] * count
    while any(cursors[p] < len(per_inst[p]) for p in range(count)):
        p = rng.choice([q for q in range(count) if cursors[q] < len(per_inst[q])])
        events.append(per_inst[p][cursors[p]])
        cursors[p] += 1
    return ns, sks, pks, events


class OracleCoinEngine:
    """CPU stand-in for GpuCoinEngine on the oracle (tests only)."""

    def __init__(self, pk_set, sk=None, variant: str = tc.DEFAULT_DIGEST):
        self.pk_set = pk_set
        self.n_keys = None
        self.sk = sk
        self.variant = variant

    def prepare(self, nonces):
        self.nonces = [bytes(x) for x in nonces]
        self.h = [tc.hash_g2(x, self.variant) for x in self.nonces]

    def sign(self):
        out = np.zeros((len(self.nonces), 96), dtype=np.uint8)
        for k, x in enumerate(self.nonces):
            out[k] = np.frombuffer(bls.g2_compress(tc.sign(self.sk, x, self.variant, hash_pt=self.h[k])), dtype=np.uint8)
        return out

    def verify(self, sigs, present):
        count, n, _ = sigs.shape
        st = np.full((count, n), SHARE_ABSENT, dtype=np.uint8)
        self.pts = {}
        for inst in range(count):
            for i in range(n):
                if not present[inst, i]:
                    continue
                try:
                    pt = bls.g2_decompress(sigs[inst, i].tobytes())
                except ValueError:
                    st[inst, i] = SHARE_UNDECODABLE
                    continue
                ok = tc.verify_sig(self.pk_set.public_key_share(i), pt, self.nonces[inst], self.variant, hash_pt=self.h[inst])
                st[inst, i] = SHARE_VALID if ok else SHARE_INVALID
                if ok:
                    self.pts[(inst, i)] = pt
        self.st = st
        return st

    def combine(self, use, t):
        count, n = use.shape
        status = np.zeros(count, dtype=np.int32)
        ok = np.zeros(count, dtype=bool)
        par = np.zeros(count, dtype=bool)
        for inst in range(count):
            shares = [(i, self.pts[(inst, i)]) for i in range(n) if use[inst, i] and self.st[inst, i] == SHARE_VALID]
            if len(shares) < t:
                status[inst] = -3
                continue
            sig = tc.combine_signatures(self.pk_set, shares)
            ok[inst] = tc.verify_sig(self.pk_set.public_key(), sig, self.nonces[inst], self.variant, hash_pt=self.h[inst])
            par[inst] = tc.parity(sig)
        return status, ok, par


def check_against_oracle(res, node):
    assert res.faults == node.faults
    assert res.errors == node.errors
    assert res.outputs == node.outputs
    assert res.combines == node.combines
    assert [(i, bytes(s)) for i, s in res.sent] == [(i, bls.g2_compress(p)) for i, p in node.sent]
