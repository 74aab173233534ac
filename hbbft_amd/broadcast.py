"""Batched replay of Broadcast (``src/broadcast.rs``) for all N instances of one epoch at one node.

The reference runs one Broadcast state machine per proposer and handles Value / Echo / Ready
messages one at a time, validating each proof (a full leaf hash plus the Merkle path) and decoding
(reconstruct + tree rebuild) whenever ``compute_output``'s conditions hold (broadcast.rs:407-551).
This host-side driver gives the same FaultLog, errors, outgoing messages and outputs, in the same
order, with the hashing and coding batched over the whole epoch on the GPU:

1. our own proposal (``handle_input`` -> ``send_shards``, :275-284, :332-404): frame on the host,
   then ``hbx_rs_encode_d`` + ``hbx_merkle_build_d`` + ``hbx_merkle_proofs_d`` -- one Value proof
   per node;
2. every proof the state machines would validate (Values from the proposer against our index,
   every Echo against its sender, :430, :451) goes into one ``hbx_merkle_validate_d`` call per
   distinct value length; validation is deterministic, so doing it early changes no result;
3. the messages are replayed in arrival order through the reference's control flow with those
   bits standing in for ``validate_proof``; each time ``compute_output`` would decode, the
   attempt (root, Echo senders holding that root) is recorded instead.  A decode result only sets
   ``decided`` (and the output): sending Echo / Ready and every fault are independent of it, so
   the replay of everything else does not wait for decodes;
4. the attempts are decoded in two waves with ``hbx_broadcast_decode_leaves_d`` (each wave one
   call per shard length): first every instance's first attempt, then all remaining distinct
   attempts of the instances whose first decode failed -- a failed decode is retried with the
   Echo values held at each later trigger, exactly as ``compute_output`` does, and an attempt
   identical to a failed one is not decoded again.  The decode takes the present shards' leaf
   digests from their validated Echo proofs (validation proved them equal to the digests of the
   values), so only the reconstructed shards are hashed.

Message model: see ``oracle/broadcast.py`` (the message-at-a-time restatement this is tested
against).  A proof is the wire ``merkle::Proof``: ``{"root_hash": 32 B, "lemma": [(node_hash,
("L"|"R", sibling) | None), ...] root first, "value": index byte + shard}``.

Limits (documented divergences for malformed input only): a lemma deeper than 16 levels (the
engine's proof layout; an honest tree over N <= 256 leaves is at most 8 deep) is treated as an
invalid proof, as is an empty value (the reference would panic indexing ``value[0]``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

RECEIVED_VALUE_FROM_NON_PROPOSER = "ReceivedValueFromNonProposer"
INVALID_PROOF = "InvalidProof"
UNKNOWN_SENDER = "UnknownSender"
NO_SUCH_BROADCAST_INSTANCE = "NoSuchBroadcastInstance"

MAX_LEMMA_DEPTH = 16


def num_faulty(n: int) -> int:
    """NetworkInfo::num_faulty (messaging.rs:258)."""
    return (n - 1) // 3


def coding_counts(n: int) -> Tuple[int, int]:
    """(data, parity) shard counts = (N - 2f, 2f) (broadcast.rs:310-311)."""
    f = num_faulty(n)
    return n - 2 * f, 2 * f


# ---------------------------------------------------------------------------------------------
# Wire-format proofs <-> the engine's flattened layout (include/hbx.h hbx_merkle_validate_d)
# ---------------------------------------------------------------------------------------------
def proof_shape_ok(p) -> bool:
    """Structural checks Proof::validate implies: 32-byte digests, a sibling on every level but the
    leaf's, a non-empty value, depth within the engine's layout."""
    lem = p.get("lemma") or []
    if not lem or len(lem) - 1 > MAX_LEMMA_DEPTH or len(p.get("value", b"")) == 0:
        return False
    if len(p.get("root_hash", b"")) != 32:
        return False
    for q, (h, sib) in enumerate(lem):
        if len(h) != 32:
            return False
        last = q == len(lem) - 1
        if last != (sib is None):
            return False
        if sib is not None and (sib[0] not in ("L", "R") or len(sib[1]) != 32):
            return False
    return True


def flatten_proofs(proofs, nodes) -> Tuple[np.ndarray, ...]:
    """Proofs of one value length -> (values, node_hash, sib_hash, sides, depth, root, sender)."""
    P = len(proofs)
    vlen = len(proofs[0]["value"])
    vals = np.zeros((P, vlen), dtype=np.uint8)
    nh = np.zeros((P, 17, 32), dtype=np.uint8)
    sh = np.zeros((P, 16, 32), dtype=np.uint8)
    sides = np.zeros(P, dtype=np.uint32)
    depth = np.zeros(P, dtype=np.uint32)
    root = np.zeros((P, 32), dtype=np.uint8)
    for j, p in enumerate(proofs):
        vals[j] = np.frombuffer(bytes(p["value"]), dtype=np.uint8)
        lem = p["lemma"]
        depth[j] = len(lem) - 1
        for lv, (h, sib) in enumerate(lem):
            nh[j, lv] = np.frombuffer(bytes(h), dtype=np.uint8)
            if sib is not None:
                sh[j, lv] = np.frombuffer(bytes(sib[1]), dtype=np.uint8)
                if sib[0] == "L":
                    sides[j] |= np.uint32(1 << lv)
        root[j] = np.frombuffer(bytes(p["root_hash"]), dtype=np.uint8)
    return vals, nh, sh, sides, depth, root, np.asarray(nodes, dtype=np.uint32)


def unflatten_proof(value: bytes, nh: np.ndarray, sh: np.ndarray, sides: int, depth: int, root: np.ndarray):
    lemma = []
    for lv in range(depth):
        lemma.append((nh[lv].tobytes(), ("L" if (sides >> lv) & 1 else "R", sh[lv].tobytes())))
    lemma.append((nh[depth].tobytes(), None))
    return {"root_hash": root.tobytes(), "lemma": lemma, "value": bytes(value)}


# ---------------------------------------------------------------------------------------------
# The engine: hbx calls on the GPU
# ---------------------------------------------------------------------------------------------
class GpuBroadcastEngine:
    """The three batched operations the replay needs, through ``hbx.Context`` (torch tensors are
    the HBM buffers; torch is plumbing only)."""

    def __init__(self, ctx, merkle_variant: int = 0, stream=None):
        import torch

        self.torch = torch
        self.ctx = ctx
        self.stream = stream
        ctx.set_merkle_digest(merkle_variant)

    def _dev(self, a):
        return self.torch.from_numpy(np.ascontiguousarray(a)).cuda(self.ctx.device)

    def send_shards(self, value: bytes, n: int) -> List[dict]:
        """broadcast.rs:332-404 for one proposal: Value proof per node, index order."""
        torch = self.torch
        k, m = coding_counts(n)
        framed = len(value).to_bytes(4, "big") + bytes(value)
        L = -(-len(framed) // k)
        buf = np.zeros((1, n, L), dtype=np.uint8)
        buf.reshape(-1)[: len(framed)] = np.frombuffer(framed, dtype=np.uint8)
        d = self._dev(buf)
        if m:
            self.ctx.rs_encode_d(d, k, m, stream=self.stream)
        cnt = self.ctx.merkle_node_count(n)
        dev = d.device
        nodes = torch.zeros((1, cnt, 32), dtype=torch.uint8, device=dev)
        self.ctx.merkle_build_d(d, nodes, stream=self.stream)
        req = self._dev(np.array([(0, j) for j in range(n)], dtype=np.uint32))
        nh = torch.zeros((n, 17, 32), dtype=torch.uint8, device=dev)
        sh = torch.zeros((n, 16, 32), dtype=torch.uint8, device=dev)
        sides = torch.zeros(n, dtype=torch.int32, device=dev)
        depth = torch.zeros(n, dtype=torch.int32, device=dev)
        root = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
        self.ctx.merkle_proofs_d(nodes, n, req, nh, sh, sides, depth, root, stream=self.stream)
        torch.cuda.synchronize(dev)
        shards = d.cpu().numpy()[0]
        nh, sh, root = nh.cpu().numpy(), sh.cpu().numpy(), root.cpu().numpy()
        sides, depth = sides.cpu().numpy().view(np.uint32), depth.cpu().numpy()
        return [unflatten_proof(bytes([i & 0xFF]) + shards[i].tobytes(), nh[i], sh[i], int(sides[i]), int(depth[i]), root[i])
                for i in range(n)]

    def validate(self, proofs, nodes, n: int) -> np.ndarray:
        """Broadcast::validate_proof(p, node) for each (p, node): one engine call per value length."""
        torch = self.torch
        out = np.zeros(len(proofs), dtype=bool)
        groups: Dict[int, List[int]] = {}
        for q, p in enumerate(proofs):
            groups.setdefault(len(p["value"]), []).append(q)
        for _, idx in sorted(groups.items()):
            arrs = flatten_proofs([proofs[q] for q in idx], [nodes[q] for q in idx])
            d = [self._dev(a) for a in arrs]
            valid = torch.zeros(len(idx), dtype=torch.uint8, device=d[0].device)
            self.ctx.merkle_validate_d(*d, n, valid, stream=self.stream)
            torch.cuda.synchronize(d[0].device)
            out[idx] = valid.cpu().numpy().astype(bool)
        return out

    def decode(self, attempts, n: int) -> List[Optional[bytes]]:
        """decode_from_shards for each attempt = (leaf values [n] (bytes|None), leaf digests [n],
        root): the value or None.  One engine call per shard length."""
        torch = self.torch
        k, m = coding_counts(n)
        out: List[Optional[bytes]] = [None] * len(attempts)
        groups: Dict[int, List[int]] = {}
        for q, (vals, _, _) in enumerate(attempts):
            lens = {len(v) for v in vals if v is not None}
            if len(lens) != 1 or 0 in lens:
                continue  # rse: IncorrectShardSize / EmptyShard (or nothing present) -> None
            if 1 in lens:
                # leaves that are only the index byte: reconstruct and the tree rebuild may run, but
                # the glued data has k * 0 < 4 bytes, so glue_shards returns None (broadcast.rs:697-707)
                continue
            groups.setdefault(lens.pop(), []).append(q)
        for vlen, idx in sorted(groups.items()):
            L = vlen - 1  # the index byte is implied by the position (validate_proof checked it)
            inst = len(idx)
            shards = np.zeros((inst, n, L), dtype=np.uint8)
            present = np.zeros((inst, n), dtype=np.uint8)
            leaf = np.zeros((inst, n, 32), dtype=np.uint8)
            roots = np.zeros((inst, 32), dtype=np.uint8)
            for r, q in enumerate(idx):
                vals, digests, root = attempts[q]
                for i, v in enumerate(vals):
                    if v is not None:
                        shards[r, i] = np.frombuffer(bytes(v), dtype=np.uint8, offset=1)
                        present[r, i] = 1
                        leaf[r, i] = np.frombuffer(bytes(digests[i]), dtype=np.uint8)
                roots[r] = np.frombuffer(bytes(root), dtype=np.uint8)
            d_sh = self._dev(shards)
            dev = d_sh.device
            d_out = torch.zeros((inst, max(k * L, 4)), dtype=torch.uint8, device=dev)
            d_len = torch.zeros(inst, dtype=torch.int64, device=dev)
            d_st = torch.zeros(inst, dtype=torch.int32, device=dev)
            self.ctx.broadcast_decode_leaves_d(d_sh, self._dev(present), self._dev(leaf), self._dev(roots), k, m, d_out,
                                               d_len, d_st, stream=self.stream)
            torch.cuda.synchronize(dev)
            st, ln, ob = d_st.cpu().numpy(), d_len.cpu().numpy(), d_out.cpu().numpy()
            for r, q in enumerate(idx):
                if st[r] == 0:
                    out[q] = ob[r, : int(ln[r])].tobytes()
        return out


# ---------------------------------------------------------------------------------------------
# The replay
# ---------------------------------------------------------------------------------------------
@dataclass
class BroadcastResult:
    faults: List[Tuple[int, str]] = field(default_factory=list)  # FaultLog entries, in order
    errors: List[Tuple[int, str]] = field(default_factory=list)  # handle_message -> Err
    sent: List[tuple] = field(default_factory=list)  # (proposer, "value"|"echo"|"ready", target|root)
    outputs: List[Tuple[int, bytes]] = field(default_factory=list)  # (proposer, value) in decision order
    decode_attempts: List[Tuple[int, bytes, bool]] = field(default_factory=list)  # as compute_output ran them
    value_proofs: Dict[int, dict] = field(default_factory=dict)  # our proposal's Value proof per node
    proof_valid: List[Optional[bool]] = field(default_factory=list)  # per event: validate_proof, if asked
    engine_decodes: int = 0  # decodes the engine ran (distinct attempts of the waves)


class _Inst:
    __slots__ = ("proposer", "echo_sent", "ready_sent", "echos", "readys", "attempts")

    def __init__(self, proposer):
        self.proposer = proposer
        self.echo_sent = False
        self.ready_sent = False
        self.echos: Dict[int, Tuple[bytes, int]] = {}  # sender -> (root, proof id)
        self.readys: Dict[int, bytes] = {}
        self.attempts: List[Tuple[int, bytes, Tuple[int, ...]]] = []  # (seq, root, senders)


class BroadcastReplay:
    """All N Broadcast instances of one epoch at node ``me`` over a batch engine."""

    def __init__(self, engine, n: int, me: int):
        self.engine = engine
        self.n = n
        self.f = num_faulty(n)
        self.k, self.m = coding_counts(n)
        self.me = me

    def run(self, events) -> BroadcastResult:
        events = list(events)
        n, me = self.n, self.me
        res = BroadcastResult(proof_valid=[None] * len(events))
        # 1. our own proposal
        own_proofs = None
        inputs = [k for k, ev in enumerate(events) if ev[0] == "input"]
        if len(inputs) > 1:
            raise ValueError("one input per Broadcast instance")
        if inputs:
            own_proofs = self.engine.send_shards(bytes(events[inputs[0]][1]), n)
        # 2. every proof a state machine may validate, in one batch
        proofs, nodes, where = [], [], []  # where: event index (or -1 for our own Value)
        if own_proofs is not None:
            proofs.append(own_proofs[me])
            nodes.append(me)
            where.append(-1)
        for k, ev in enumerate(events):
            if ev[0] not in ("value", "echo"):
                continue
            _, sender, proposer, p = ev
            if not (0 <= proposer < n and 0 <= sender < n):
                continue
            if ev[0] == "value" and sender != proposer:
                continue  # rejected before validation (:409-418)
            proofs.append(p)
            nodes.append(me if ev[0] == "value" else sender)
            where.append(k)
        shape = [proof_shape_ok(p) for p in proofs]
        valid = np.zeros(len(proofs), dtype=bool)
        sel = [q for q in range(len(proofs)) if shape[q]]
        if sel:
            valid[sel] = self.engine.validate([proofs[q] for q in sel], [nodes[q] for q in sel], n)
        ok_of = {w: bool(valid[q]) for q, w in enumerate(where)}
        pid_of = {w: q for q, w in enumerate(where)}
        for w, ok in ok_of.items():
            if w >= 0:
                res.proof_valid[w] = ok
        # 3. the control flow, message by message; decodes recorded as attempts
        insts = [_Inst(p) for p in range(n)]
        seq = [0]

        def count_echos(b, h):
            return sum(1 for r, _ in b.echos.values() if r == h)

        def count_readys(b, h):
            return sum(1 for x in b.readys.values() if x == h)

        def compute_output(b, h):
            if count_readys(b, h) <= 2 * self.f or count_echos(b, h) < self.k:
                return
            senders = tuple(i for i in sorted(b.echos) if b.echos[i][0] == h)
            b.attempts.append((seq[0], h, senders))
            seq[0] += 1

        def send_ready(b, h):
            b.ready_sent = True
            res.sent.append((b.proposer, "ready", h))
            handle_ready(b, me, h)

        def handle_ready(b, sender, h):
            if sender in b.readys:
                return
            b.readys[sender] = h
            if count_readys(b, h) == self.f + 1 and not b.ready_sent:
                send_ready(b, h)
            compute_output(b, h)

        def handle_echo(b, sender, key):
            if sender in b.echos:
                return
            if not ok_of[key]:
                res.faults.append((sender, INVALID_PROOF))
                return
            h = bytes(proofs[pid_of[key]]["root_hash"])
            b.echos[sender] = (h, pid_of[key])
            if b.ready_sent or count_echos(b, h) < n - self.f:
                compute_output(b, h)
                return
            send_ready(b, h)

        def handle_value(b, sender, key):
            if sender != b.proposer:
                res.faults.append((sender, RECEIVED_VALUE_FROM_NON_PROPOSER))
                return
            if b.echo_sent:
                return
            if not ok_of[key]:
                res.faults.append((sender, INVALID_PROOF))
                return
            b.echo_sent = True  # send_echo (:494-504)
            res.sent.append((b.proposer, "echo", bytes(proofs[pid_of[key]]["root_hash"])))
            handle_echo(b, me, key)

        for k, ev in enumerate(events):
            if ev[0] == "input":
                for i in range(n):
                    if i != me:
                        res.sent.append((me, "value", i))
                        res.value_proofs[i] = own_proofs[i]
                handle_value(insts[me], me, -1)
                continue
            _, sender, proposer, payload = ev
            if not 0 <= proposer < n:
                res.errors.append((sender, NO_SUCH_BROADCAST_INSTANCE))
                continue
            if not 0 <= sender < n:
                res.errors.append((sender, UNKNOWN_SENDER))
                continue
            b = insts[proposer]
            if ev[0] == "value":
                handle_value(b, sender, k)
            elif ev[0] == "echo":
                handle_echo(b, sender, k)
            elif ev[0] == "ready":
                handle_ready(b, sender, bytes(payload))
            else:
                raise ValueError(ev[0])
        # 4. decode waves
        decided = self._decode_waves(insts, proofs, res)
        # outputs and the attempts compute_output actually ran, in the reference's order
        ran = []
        for b in insts:
            stop = decided.get(b.proposer)
            for a in b.attempts:
                if stop is not None and a[0] > stop[0]:
                    break
                ran.append((a[0], b.proposer, a[1], stop is not None and a[0] == stop[0]))
        ran.sort()
        res.decode_attempts = [(p, h, ok) for _, p, h, ok in ran]
        res.outputs = [(p, decided[p][1]) for _, p, _, ok in ran if ok]
        return res

    def _decode_waves(self, insts, proofs, res) -> Dict[int, Tuple[int, bytes]]:
        """proposer -> (seq of the first successful attempt, value)."""
        n = self.n
        cache: Dict[Tuple[int, bytes, Tuple[int, ...]], Optional[bytes]] = {}

        def build(b, h, senders):
            vals: List[Optional[bytes]] = [None] * n
            digests: List[Optional[bytes]] = [None] * n
            for i in senders:
                p = proofs[b.echos[i][1]]
                vals[i] = bytes(p["value"])
                digests[i] = bytes(p["lemma"][-1][0])  # the leaf digest validation checked
            return vals, digests, h

        def run(batch):
            todo = [key for key in dict.fromkeys(batch) if key not in cache]
            if todo:
                got = self.engine.decode([build(insts[p], h, s) for p, h, s in todo], n)
                res.engine_decodes += len(todo)
                for key, v in zip(todo, got):
                    cache[key] = v

        first = [(b.proposer, b.attempts[0][1], b.attempts[0][2]) for b in insts if b.attempts]
        run(first)
        rest = [(b.proposer, a[1], a[2]) for b in insts if b.attempts and cache[(b.proposer,) + b.attempts[0][1:]] is None
                for a in b.attempts[1:]]
        run(rest)
        decided = {}
        for b in insts:
            for a in b.attempts:
                v = cache[(b.proposer, a[1], a[2])]
                if v is not None:
                    decided[b.proposer] = (a[0], v)
                    break
        return decided
