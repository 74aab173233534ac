"""Batched replay of HoneyBadger's threshold-decryption sub-path for one node-epoch.

The reference handles decryption shares one message at a time (``src/honey_badger/
honey_badger.rs``: ``handle_decryption_share_message`` :186-217, ``send_decryption_shares``
:351-391, ``verify_pending_decryption_shares`` :422-444, ``try_decrypt_proposer_contribution``
:315-349).  This host-side driver gives the same FaultLog, in the same order, and the same Batch,
with ONE engine pass over the whole epoch instead of one pairing check per message:

1. the CommonSubset output (the accepted ciphertexts) goes through ``hbx_prepare_ciphertexts``
   (hash_g1_g2 hoisted per proposer, ``Ciphertext::verify``) -> one ``HBX_CT_*`` status each;
2. every DecryptionShare message of the epoch, before or after the ciphertexts, goes into one
   ``hbx_verify_dec_shares`` call (a second call per extra message of the same (proposer, sender)
   pair, which only a Byzantine sender produces) -> one ``HBX_SHARE_*`` status per message;
3. the messages are then replayed in arrival order through the reference's control flow, with the
   statuses standing in for the pairing checks: verification is deterministic, so verifying a
   share early changes no result, only when the work is done;
4. the plaintexts come from ``hbx_combine_decrypt`` (first t valid shares by index; any t valid
   shares interpolate to the same point, so the bytes equal the reference's, whichever t shares
   it had when it crossed the threshold).

Message model: see ``oracle/honey_badger.py`` (the message-at-a-time restatement this is tested
against): ``("share", sender, proposer, share48)`` and ``("acs", {proposer: (u48, v, w96)})``.
A node does not receive its own share messages (it inserts its own share itself, :394-418).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from .hbx import CT_INVALID, CT_UNDECODABLE, CT_VALID, SHARE_INVALID, SHARE_UNDECODABLE

UNVERIFIED_DECRYPTION_SHARE_SENDER = "UnverifiedDecryptionShareSender"
INVALID_CIPHERTEXT = "InvalidCiphertext"
SHARE_DECRYPTION_FAILED = "ShareDecryptionFailed"
UNKNOWN_SENDER = "UnknownSender"


@dataclass
class EpochResult:
    faults: List[Tuple[int, str]] = field(default_factory=list)  # FaultLog entries, in order
    errors: List[Tuple[int, str]] = field(default_factory=list)  # handle_message -> Err
    batch: Optional[Dict[int, bytes]] = None  # proposer -> contribution, once the epoch output
    decrypt_errors: List[int] = field(default_factory=list)  # proposers whose decrypt failed (:345)
    ct_status: Dict[int, int] = field(default_factory=dict)  # proposer -> HBX_CT_*
    share_status: List[Optional[int]] = field(default_factory=list)  # per event: HBX_SHARE_* or None


class EpochReplay:
    """One node-epoch of the decryption sub-path over an ``hbx.Context``.

    ``ctx`` must hold the era's key shares (``set_pk_shares``, n keys); ``sk_me`` is this node's
    32-byte secret key share, installed with ``set_own_share`` so the engine computes our own
    decryption shares (``decrypt_share_no_verify``, :403) and checks the ciphertexts through
    them."""

    def __init__(self, ctx, n: int, me: int, sk_me: bytes):
        self.ctx = ctx
        self.n = n
        self.f = (n - 1) // 3  # NetworkInfo::num_faulty, messaging.rs:258
        # PublicKeySet::decrypt needs threshold + 1 = f + 1 shares (the key set's threshold is f)
        self.t = self.f + 1
        self.me = me
        self.sk_me = bytes(sk_me)

    # ------------------------------------------------------------------------------------------
    def _engine(self, events, acs_pos):
        """Steps 1-2: ciphertext statuses and one status per share message of an ACS proposer."""
        cs_output = events[acs_pos][1]
        props = sorted(cs_output)
        col = {pid: j for j, pid in enumerate(props)}
        p, n = len(props), self.n
        self.ctx.set_own_share(self.me, self.sk_me)
        self.ctx.prepare_ciphertexts([cs_output[pid] for pid in props])
        ct_status = self.ctx.ct_status(p)
        # layer L holds the L-th message of every (proposer, sender) pair
        layers: List[Dict[Tuple[int, int], int]] = []
        seen: Dict[Tuple[int, int], int] = {}
        for k, ev in enumerate(events):
            if ev[0] != "share":
                continue
            _, sender, pid, _ = ev
            if sender >= n or pid not in col:
                continue
            if sender == self.me:
                raise ValueError("a node does not receive its own DecryptionShare messages")
            key = (col[pid], sender)
            L = seen.get(key, 0)
            seen[key] = L + 1
            if L == len(layers):
                layers.append({})
            layers[L][key] = k
        status: Dict[int, int] = {}
        for layer in layers or [{}]:
            shares = np.zeros((p, n, 48), dtype=np.uint8)
            present = np.zeros((p, n), dtype=bool)
            for (j, i), k in layer.items():
                shares[j, i] = np.frombuffer(bytes(events[k][3]), dtype=np.uint8)
                present[j, i] = True
            self.ctx.verify_dec_shares(shares, present)
            st = self.ctx.share_status(p, n)
            for (j, i), k in layer.items():
                status[k] = int(st[j, i])
        return props, {pid: int(ct_status[j]) for j, pid in enumerate(props)}, status, layers

    def run(self, events) -> EpochResult:
        events = list(events)
        res = EpochResult(share_status=[None] * len(events))
        acs = [k for k, ev in enumerate(events) if ev[0] == "acs"]
        if len(acs) > 1:
            raise ValueError("one CommonSubset output per epoch")
        acs_pos = acs[0] if acs else None
        props, ct_st, status, layers = ([], {}, {}, []) if acs_pos is None else self._engine(events, acs_pos)
        res.ct_status = ct_st
        for k, s in status.items():
            res.share_status[k] = s

        valid_cts: Optional[List[int]] = None  # proposers with a verified ciphertext, after the ACS
        received: Dict[int, Dict[int, int]] = {}  # proposer -> sender -> event index (-1 = own share)
        decrypted: set = set()
        done = False

        def try_output():
            nonlocal done
            if done or valid_cts is None:
                return
            ok = True
            for pid in valid_cts:  # all(): stops at the first proposer still short of shares
                if pid in decrypted:
                    continue
                if len(received.get(pid, {})) <= self.f:
                    ok = False
                    break
                decrypted.add(pid)
            if ok:
                done = True

        for k, ev in enumerate(events):
            if done:
                break  # messages of a past epoch are ignored (:68-76)
            if ev[0] == "share":
                _, sender, pid, _ = ev
                if sender >= self.n:
                    res.errors.append((sender, UNKNOWN_SENDER))
                    continue
                st = status.get(k)
                if st == SHARE_UNDECODABLE:
                    continue  # serde rejects the message before HoneyBadger sees it
                if valid_cts is not None and pid in valid_cts and st == SHARE_INVALID:
                    res.faults.append((sender, UNVERIFIED_DECRYPTION_SHARE_SENDER))
                    continue
                received.setdefault(pid, {})[sender] = k
                try_output()
            else:  # the CommonSubset output: send_decryption_shares
                valid_cts = []
                for pid in props:
                    if ct_st[pid] == CT_UNDECODABLE:
                        res.faults.append((pid, INVALID_CIPHERTEXT))
                        continue
                    if ct_st[pid] == CT_INVALID:
                        res.faults.append((pid, SHARE_DECRYPTION_FAILED))
                        continue
                    assert ct_st[pid] == CT_VALID
                    pending = received.get(pid, {})
                    for sender in sorted(pending):
                        if status.get(pending[sender]) == SHARE_INVALID:
                            res.faults.append((sender, UNVERIFIED_DECRYPTION_SHARE_SENDER))
                            del pending[sender]
                    received.setdefault(pid, {})[self.me] = -1  # our own share
                    valid_cts.append(pid)
                try_output()

        if done:
            res.batch = self._decrypt(events, props, received, decrypted, len(layers) > 1, res.decrypt_errors)
        return res

    def _decrypt(self, events, props, received, decrypted, relayer: bool, errors: List[int]) -> Dict[int, bytes]:
        """Step 4.  With several messages per pair, verify the final share set once more so the
        engine's combine reads exactly the shares the node ended up holding."""
        p, n = len(props), self.n
        if relayer:
            shares = np.zeros((p, n, 48), dtype=np.uint8)
            present = np.zeros((p, n), dtype=bool)
            for j, pid in enumerate(props):
                for sender, k in received.get(pid, {}).items():
                    if k >= 0:
                        shares[j, sender] = np.frombuffer(bytes(events[k][3]), dtype=np.uint8)
                        present[j, sender] = True
            self.ctx.verify_dec_shares(shares, present)
        plains, st = self.ctx.combine_decrypt(self.t)
        out = {}
        for j, pid in enumerate(props):
            if pid in decrypted:
                if st[j] != 0:
                    # PublicKeySet::decrypt returned Err: the reference only logs it (:345) and the
                    # proposer is left out of the batch
                    errors.append(pid)
                    continue
                out[pid] = plains[j]
        return out
