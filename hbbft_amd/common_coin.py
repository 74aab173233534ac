"""Batched replay of the Common Coin (``src/common_coin.rs``) for every coin instance of a round at
one node.

The reference runs one ``CommonCoin`` per Agreement instance and handles its signature shares one
message at a time: each share is verified on arrival (``PublicKeyShare::verify``, :151), and as
soon as the node has had its input and holds more than f valid shares it combines them
(``combine_signatures``, :190), checks the result against the master key (:196) and outputs the
parity (:173), ignoring every later message (:105-110).  This host-side driver gives the same
FaultLog, errors, messages and outputs, in the same order, with ONE engine pass per step:

1. ``hbx_prepare_nonces``: hash_g2 of every instance's nonce, once;
2. our own share of every instance we input to: one ``hbx_sign`` call;
3. every signature share of the round -- received messages and our own shares, in arrival order
   -- in one ``hbx_verify_sig_shares_d`` call (a second call per extra message of the same
   (instance, sender) pair, which only a Byzantine sender produces) -> one HBX_SHARE_* status per
   message; verification is deterministic, so verifying early changes no result;
4. the messages are replayed in arrival order through the reference's control flow with those
   statuses; each time ``try_output`` would combine, the set of shares the instance holds at that
   moment is recorded and the instance is taken to terminate;
5. the recorded sets are combined in one ``hbx_combine_signatures_d`` call, restricted to exactly
   those shares (``d_use``); a combination that fails the master check (``VerificationFailed``:
   the reference keeps the instance open and retries on a later share) is remembered and the
   replay runs again, so the retries happen exactly where the reference would run them.

Message model: see ``oracle/common_coin.py`` (the message-at-a-time restatement this is tested
against): ``("input", inst)`` and ``("share", sender, inst, sig96)``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from .hbx import SHARE_INVALID, SHARE_UNDECODABLE, SHARE_VALID

UNVERIFIED_SIGNATURE_SHARE_SENDER = "UnverifiedSignatureShareSender"
UNKNOWN_SENDER = "UnknownSender"
VERIFICATION_FAILED = "VerificationFailed"
COMBINE_FAILED = "CombineAndVerifySigCrypto"


@dataclass
class CoinResult:
    faults: List[Tuple[int, str]] = field(default_factory=list)  # FaultLog entries, in order
    errors: List[Tuple[Optional[int], str]] = field(default_factory=list)  # (sender, error) in order
    sent: List[Tuple[int, bytes]] = field(default_factory=list)  # (inst, our share) sent to all
    outputs: List[Tuple[int, bool]] = field(default_factory=list)  # (inst, parity) in output order
    combines: List[Tuple[int, Tuple[int, ...], bool]] = field(default_factory=list)  # as try_output ran
    share_status: List[Optional[int]] = field(default_factory=list)  # per event: HBX_SHARE_* or None
    engine_combines: int = 0  # engine combine calls (1 unless a combination failed)


class GpuCoinEngine:
    """The batched coin operations on the GPU through ``hbx.Context`` (torch tensors are the HBM
    buffers; torch is plumbing only).  The context holds the era's key shares
    (``set_pk_shares``)."""

    def __init__(self, ctx, master_pk48: bytes, sk32: Optional[bytes] = None, stream=None):
        import torch

        self.torch = torch
        self.ctx = ctx
        self.master_pk48 = bytes(master_pk48)
        self.sk32 = None if sk32 is None else bytes(sk32)
        self.stream = stream
        self.count = 0

    def prepare(self, nonces):
        self.ctx.prepare_nonces([bytes(x) for x in nonces], hashes=False)
        self.count = len(nonces)

    def sign(self) -> np.ndarray:
        """Our share of every prepared nonce -> uint8[count, 96]."""
        sk = np.frombuffer(self.sk32, dtype=np.uint8).reshape(1, 32)
        return self.ctx.sign(sk)[:, 0]

    def verify(self, sigs: np.ndarray, present: np.ndarray) -> np.ndarray:
        torch = self.torch
        count, n, _ = sigs.shape
        dev = torch.device("cuda", self.ctx.device)
        d_sig = torch.from_numpy(np.ascontiguousarray(sigs)).to(dev)
        d_pres = torch.from_numpy(np.ascontiguousarray(present, dtype=np.uint8)).to(dev)
        d_st = torch.zeros((count, n), dtype=torch.uint8, device=dev)
        self.ctx.verify_sig_shares_d(d_sig, d_pres, d_st, stream=self.stream)
        return d_st.cpu().numpy()

    def combine(self, use: np.ndarray, t: int):
        """Over the shares of the last ``verify`` call restricted to ``use`` -> (status int32[count],
        master_ok bool[count], parity bool[count])."""
        torch = self.torch
        count = use.shape[0]
        dev = torch.device("cuda", self.ctx.device)
        d_use = torch.from_numpy(np.ascontiguousarray(use, dtype=np.uint8)).to(dev)
        d_st = torch.zeros(count, dtype=torch.int32, device=dev)
        d_ok = torch.zeros(count, dtype=torch.uint8, device=dev)
        d_par = torch.zeros(count, dtype=torch.uint8, device=dev)
        self.ctx.combine_signatures_d(self.master_pk48, t, d_use, None, d_st, d_ok, d_par, stream=self.stream)
        return d_st.cpu().numpy(), d_ok.cpu().numpy().astype(bool), d_par.cpu().numpy().astype(bool)


class _Inst:
    __slots__ = ("had_input", "terminated", "received")

    def __init__(self):
        self.had_input = False
        self.terminated = False
        self.received: Dict[int, int] = {}  # sender -> message id (BTreeMap<N, SignatureShare>)


class CoinReplay:
    """Every CommonCoin instance of a round at node ``me`` (None: an observer, not a validator)."""

    def __init__(self, engine, n: int, me: Optional[int]):
        self.engine = engine
        self.n = n
        self.f = (n - 1) // 3  # NetworkInfo::num_faulty, messaging.rs:258
        self.t = self.f + 1    # combine_signatures needs threshold + 1 shares
        self.me = me

    def run(self, nonces, events) -> CoinResult:
        events = list(events)
        count, n = len(nonces), self.n
        self.engine.prepare(nonces)
        inputs = {ev[1] for ev in events if ev[0] == "input"}
        own = self.engine.sign() if (self.me is not None and inputs) else None
        # the share messages: received ones and, at our first input to an instance, our own
        msgs: List[Tuple[int, int, bytes]] = []  # (inst, sender, sig96)
        msg_of_event: Dict[int, int] = {}
        seen_input = set()
        for k, ev in enumerate(events):
            if ev[0] == "input":
                inst = ev[1]
                if self.me is not None and inst not in seen_input:
                    msg_of_event[k] = len(msgs)
                    msgs.append((inst, self.me, bytes(own[inst])))
                seen_input.add(inst)
            elif ev[0] == "share":
                _, sender, inst, sig96 = ev
                msg_of_event[k] = len(msgs)
                msgs.append((inst, sender, bytes(sig96)))
            else:
                raise ValueError(ev[0])
        status, layer_of = self._verify(msgs, count)
        res_status = [None] * len(events)
        for k, m in msg_of_event.items():
            if events[k][0] == "share" and 0 <= events[k][1] < n:
                res_status[k] = int(status[m])
        # replay + combine waves until every combination the control flow runs is known
        known: Dict[Tuple[int, Tuple[Tuple[int, int], ...]], Tuple[Optional[str], bool]] = {}  # -> (error, parity)
        combines_run = 0
        while True:
            res, pending = self._replay(events, msgs, msg_of_event, status, known, count)
            if not pending:
                break
            combines_run += 1
            self._combine(pending, msgs, layer_of, known, count)
        res.share_status = res_status
        res.engine_combines = combines_run
        return res

    # ------------------------------------------------------------------------------------------
    def _verify(self, msgs, count):
        """One engine call per layer (layer L = the L-th message of each (inst, sender) pair).  A
        message from a non-validator is never verified, but whether serde would have decoded it
        decides between no reaction and UnknownSender: those go first, through columns of their
        own instance's row (only the UNDECODABLE status is used), so that the real layers are the
        last verifications the engine holds."""
        n = self.n
        unknown = [m for m, (_, sender, _) in enumerate(msgs) if not 0 <= sender < n]
        status = np.full(len(msgs), SHARE_UNDECODABLE, dtype=np.int32)
        # decode-only layers: the unknown-sender messages of each instance over columns 0..n-1
        slot: Dict[int, int] = {}
        batches: List[Dict[Tuple[int, int], int]] = []
        for m in unknown:
            inst = msgs[m][0]
            q = slot.get(inst, 0)
            slot[inst] = q + 1
            if q // n == len(batches):
                batches.append({})
            batches[q // n][(inst, q % n)] = m
        for batch in batches:
            st = self._verify_layer(batch, msgs, count)
            for key, m in batch.items():
                status[m] = SHARE_UNDECODABLE if st[key] == SHARE_UNDECODABLE else SHARE_INVALID
        layers: List[Dict[Tuple[int, int], int]] = []
        seen: Dict[Tuple[int, int], int] = {}
        layer_of = [-1] * len(msgs)
        for m, (inst, sender, _) in enumerate(msgs):
            if not 0 <= sender < n:
                continue
            key = (inst, sender)
            L = seen.get(key, 0)
            seen[key] = L + 1
            if L == len(layers):
                layers.append({})
            layers[L][key] = m
            layer_of[m] = L
        for layer in layers:
            st = self._verify_layer(layer, msgs, count)
            for key, m in layer.items():
                status[m] = st[key]
        self._last_layer = len(layers) - 1
        return status, layer_of

    def _verify_layer(self, layer, msgs, count):
        sigs = np.zeros((count, self.n, 96), dtype=np.uint8)
        present = np.zeros((count, self.n), dtype=np.uint8)
        for key, m in layer.items():
            sigs[key] = np.frombuffer(msgs[m][2], dtype=np.uint8)
            present[key] = 1
        return self.engine.verify(sigs, present)

    def _replay(self, events, msgs, msg_of_event, status, known, count):
        res = CoinResult()
        insts = [_Inst() for _ in range(count)]
        pending: Dict[int, Tuple[Tuple[int, int], ...]] = {}  # inst -> held (sender, msg id) set

        def try_output(inst, who):
            b = insts[inst]
            if not (b.had_input and len(b.received) > self.f):
                return
            held = tuple(sorted(b.received.items()))
            senders = tuple(s for s, _ in held)
            r = known.get((inst, held))
            if r is None:
                pending[inst] = held  # combined after this pass; taken to succeed meanwhile
                b.terminated = True
                return
            err, par = r
            res.combines.append((inst, senders, err is None))
            if err is not None:
                res.errors.append((who, err))
                return
            b.terminated = True
            res.outputs.append((inst, par))

        def handle_share(inst, sender, m, who):
            b = insts[inst]
            st = status[m]
            if st != SHARE_VALID:
                if st == SHARE_INVALID:
                    res.faults.append((sender, UNVERIFIED_SIGNATURE_SHARE_SENDER))
                return
            b.received[sender] = m
            try_output(inst, who)

        for k, ev in enumerate(events):
            if ev[0] == "input":
                inst = ev[1]
                b = insts[inst]
                if b.had_input:
                    continue
                b.had_input = True
                if self.me is None:
                    try_output(inst, None)
                    continue
                m = msg_of_event[k]
                # get_coin (common_coin.rs:142-146): an error from our own share's handle_share
                # drops the step with the outgoing message (the `?`); the error is our input's
                n_err = len(res.errors)
                handle_share(inst, self.me, m, None)
                if len(res.errors) == n_err:
                    res.sent.append((inst, msgs[m][2]))
            else:
                _, sender, inst, _ = ev
                b = insts[inst]
                if status[msg_of_event[k]] == SHARE_UNDECODABLE:
                    continue  # rejected by serde before CommonCoin
                if b.terminated:
                    continue  # handle_message after termination (:105-110)
                if not 0 <= sender < self.n:
                    res.errors.append((sender, UNKNOWN_SENDER))
                    continue
                handle_share(inst, sender, msg_of_event[k], sender)
        return res, pending

    def _combine(self, pending, msgs, layer_of, known, count):
        """One engine combine over the pending sets.  When every held share is in the last
        verified layer (always, unless a sender repeated itself), the combination reuses that
        verification through the use mask; otherwise the held shares are verified again as one
        layer of their own (they were verified before, so their statuses do not change)."""
        n = self.n
        last = self._last_layer
        use = np.zeros((count, n), dtype=np.uint8)
        reuse = all(layer_of[m] == last for held in pending.values() for _, m in held)
        if not reuse:
            sigs = np.zeros((count, n, 96), dtype=np.uint8)
            present = np.zeros((count, n), dtype=np.uint8)
            for inst, held in pending.items():
                for s, m in held:
                    sigs[inst, s] = np.frombuffer(msgs[m][2], dtype=np.uint8)
                    present[inst, s] = 1
            self.engine.verify(sigs, present)
            self._last_layer = -1  # the engine's last verification is no longer a layer
        for inst, held in pending.items():
            for s, _ in held:
                use[inst, s] = 1
        st, ok, par = self.engine.combine(use, self.t)
        for inst, held in pending.items():
            err = COMBINE_FAILED if st[inst] != 0 else None if ok[inst] else VERIFICATION_FAILED
            known[(inst, held)] = (err, bool(par[inst]))
