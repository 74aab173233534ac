"""Broadcast (Bracha reliable broadcast with RS + Merkle, ``src/broadcast.rs``) for all N
instances of one epoch at ONE node, one message at a time -- TEST ORACLE ONLY.

Only ``tests/`` (and fixture scripts under ``tests/golden/``) may import this.  It restates the
reference's state machine line by line, with the CPU Reed-Solomon / Merkle of
``oracle/rs_merkle.py``, so that the batched replay in ``hbbft_amd/broadcast.py`` (batched proof
validation and decodes on the GPU) can be checked to emit the same FaultLog, errors, outgoing
messages and outputs, in the same order:

* ``CommonSubset::handle_broadcast`` / ``process_broadcast`` common_subset.rs:174-220 -- a message
  for a proposer that has no instance is ``Err(NoSuchBroadcastInstance)``;
* ``Broadcast::handle_message`` broadcast.rs:286-295 -- a sender that is not a validator is
  ``Err(UnknownSender)``;
* ``handle_input`` / ``send_shards`` :275-284, :332-404 -- frame, RS encode, index bytes, Merkle
  tree, one ``Value`` proof per node; our own proof goes through ``handle_value``;
* ``handle_value`` :407-436 -- a Value from anyone but the proposer is
  ``ReceivedValueFromNonProposer``; a second Value is ignored once the Echo was sent; an invalid
  proof (``validate_proof(p, our_uid)``) is ``InvalidProof``; else ``send_echo``;
* ``handle_echo`` :439-466 -- a second Echo of a sender is ignored; ``validate_proof(p, sender)``
  or ``InvalidProof``; stored; then ``compute_output`` if Ready was sent or fewer than N - f
  Echos carry this root, else ``send_ready``;
* ``handle_ready`` :469-491 -- a second Ready of a sender is ignored; stored; f + 1 matching Readys
  and no Ready sent yet -> ``send_ready``; then ``compute_output``;
* ``send_echo`` / ``send_ready`` :494-517 -- multicast and handle our own message;
* ``compute_output`` :521-551 -- nothing once decided, or with <= 2f Readys or < k Echos for this
  root; else ``decode_from_shards`` over the Echo values carrying this root (index byte
  included): reconstruct, rebuild the tree, compare the root, glue (:660-707).  A failed decode
  leaves the instance undecided, so every later Echo / Ready that reaches ``compute_output`` with
  the conditions met tries again (with the Echo values held at that time).
* ``validate_proof`` :555-575 -- ``Proof::validate(root_hash)``, ``value[0] ==
  node_index(id)`` and ``Proof::index(N) == value[0]``.  An empty value is invalid here (the
  reference would index ``value[0]`` out of bounds and panic).

Decode detail restated from reed-solomon-erasure 3.1.0 (``reconstruct_shards``): the present
shards must all have the same, non-zero length (``IncorrectShardSize`` / ``EmptyShard``), checked
before the all-present shortcut; any error makes ``decode_from_shards`` return None (:667-670).
That error order is the crate's published code as remembered (unpinned detail); it only matters
for a Byzantine proposer whose leaves differ in length.

Message model (what crosses the wire, with node indices for ids -- BTreeMap order,
messaging.rs:246-250):
  ("input", value)                       -- our own proposal (we are its instance's proposer)
  ("value", sender, proposer, proof)     -- BroadcastMessage::Value
  ("echo",  sender, proposer, proof)     -- BroadcastMessage::Echo
  ("ready", sender, proposer, hash32)    -- BroadcastMessage::Ready
A proof is ``oracle.rs_merkle``'s dict ``{root_hash, lemma, value}``.
"""
from __future__ import annotations

from . import rs_merkle as rm

RECEIVED_VALUE_FROM_NON_PROPOSER = "ReceivedValueFromNonProposer"
INVALID_PROOF = "InvalidProof"
UNKNOWN_SENDER = "UnknownSender"
NO_SUCH_BROADCAST_INSTANCE = "NoSuchBroadcastInstance"


def reconstruct_checked(leaf_values, k: int, m: int):
    """Coding::reconstruct_shards (broadcast.rs:643-657) with rse 3.1.0's shard checks; returns the
    full list of leaves or None on any error."""
    present = [v for v in leaf_values if v is not None]
    lens = {len(v) for v in present}
    if len(lens) > 1 or 0 in lens:
        return None  # IncorrectShardSize / EmptyShard
    if m == 0:  # Coding::Trivial
        return None if len(present) < len(leaf_values) else [bytes(v) for v in leaf_values]
    try:
        return rm.ReedSolomon(k, m).reconstruct(leaf_values)
    except rm.TooFewShardsPresent:
        return None


def decode_from_shards(leaf_values, n: int, root_hash: bytes, variant: str = "sha256"):
    """broadcast.rs:660-692 (+ glue :697-707): the value, or None."""
    k, m = rm.coding_counts(n)
    leaves = reconstruct_checked(leaf_values, k, m)
    if leaves is None:
        return None
    if rm.MerkleTree(leaves, variant).root_hash() != root_hash:
        return None
    return rm.glue_shards(leaves, k)


class Instance:
    """One Broadcast instance (broadcast.rs:229-247): state for the proposal of `proposer`."""

    def __init__(self, proposer: int):
        self.proposer = proposer
        self.echo_sent = False
        self.ready_sent = False
        self.decided = False
        self.echos = {}  # sender -> proof (BTreeMap<N, Proof>)
        self.readys = {}  # sender -> hash (BTreeMap<N, Vec<u8>>)
        self.output = None


class BroadcastNode:
    """Node `me` of n validators, with one Broadcast instance per proposer (CommonSubset)."""

    def __init__(self, n: int, me: int, variant: str = "sha256"):
        self.n = n
        self.f = rm.num_faulty(n)
        self.k, self.m = rm.coding_counts(n)
        self.me = me
        self.variant = variant
        self.inst = {p: Instance(p) for p in range(n)}
        self.faults = []  # (node, FaultKind), in emission order
        self.errors = []  # (node, error): handle_message returned Err
        self.sent = []  # (proposer, "value" | "echo" | "ready", target | root hash), in order
        self.outputs = []  # (proposer, value) in decision order
        self.decode_attempts = []  # (proposer, hash, ok): every decode_from_shards call
        self.value_proofs = {}  # node -> the Value proof send_shards addressed to it
        self.outbox = []  # (target node | None = all others, event as the receiver sees it)

    # -- helpers ------------------------------------------------------------------------------
    def _validate(self, p, node: int) -> bool:
        # a lemma deeper than 16 levels is rejected (the engine's proof layout; an honest tree of
        # N <= 256 leaves is at most 8 deep): a documented divergence for malformed proofs only
        if len(p["value"]) == 0 or not p["lemma"] or len(p["lemma"]) - 1 > 16:
            return False
        return rm.validate_broadcast_proof(p, node, self.n, self.variant)

    def _count_echos(self, b: Instance, h: bytes) -> int:
        return sum(1 for p in b.echos.values() if p["root_hash"] == h)

    def _count_readys(self, b: Instance, h: bytes) -> int:
        return sum(1 for x in b.readys.values() if x == h)

    # -- handlers -------------------------------------------------------------------------------
    def handle(self, ev):
        kind = ev[0]
        if kind == "input":
            self._handle_input(ev[1])
            return
        _, sender, proposer, payload = ev
        if proposer not in self.inst:
            self.errors.append((sender, NO_SUCH_BROADCAST_INSTANCE))
            return
        if not 0 <= sender < self.n:
            self.errors.append((sender, UNKNOWN_SENDER))
            return
        b = self.inst[proposer]
        if kind == "value":
            self._handle_value(b, sender, payload)
        elif kind == "echo":
            self._handle_echo(b, sender, payload)
        elif kind == "ready":
            self._handle_ready(b, sender, bytes(payload))
        else:
            raise ValueError(kind)

    def _handle_input(self, value: bytes):
        b = self.inst[self.me]
        _, leaves, tree = rm.send_shards(bytes(value), self.n, self.variant)
        ours = None
        for i, leaf in enumerate(leaves):
            proof = tree.gen_proof(leaf)
            if i == self.me:
                ours = proof
            else:
                self.sent.append((self.me, "value", i))
                self.value_proofs[i] = proof
                self.outbox.append((i, ("value", self.me, self.me, proof)))
        self._handle_value(b, self.me, ours)

    def _handle_value(self, b: Instance, sender: int, p):
        if sender != b.proposer:
            self.faults.append((sender, RECEIVED_VALUE_FROM_NON_PROPOSER))
            return
        if b.echo_sent:
            return
        if not self._validate(p, self.me):
            self.faults.append((sender, INVALID_PROOF))
            return
        self._send_echo(b, p)

    def _handle_echo(self, b: Instance, sender: int, p):
        if sender in b.echos:
            return
        if not self._validate(p, sender):
            self.faults.append((sender, INVALID_PROOF))
            return
        h = p["root_hash"]
        b.echos[sender] = p
        if b.ready_sent or self._count_echos(b, h) < self.n - self.f:
            self._compute_output(b, h)
            return
        self._send_ready(b, h)

    def _handle_ready(self, b: Instance, sender: int, h: bytes):
        if sender in b.readys:
            return
        b.readys[sender] = h
        if self._count_readys(b, h) == self.f + 1 and not b.ready_sent:
            self._send_ready(b, h)
        self._compute_output(b, h)

    def _send_echo(self, b: Instance, p):
        b.echo_sent = True
        self.sent.append((b.proposer, "echo", p["root_hash"]))
        self.outbox.append((None, ("echo", self.me, b.proposer, p)))
        self._handle_echo(b, self.me, p)

    def _send_ready(self, b: Instance, h: bytes):
        b.ready_sent = True
        self.sent.append((b.proposer, "ready", h))
        self.outbox.append((None, ("ready", self.me, b.proposer, h)))
        self._handle_ready(b, self.me, h)

    def _compute_output(self, b: Instance, h: bytes):
        if b.decided or self._count_readys(b, h) <= 2 * self.f or self._count_echos(b, h) < self.k:
            return
        leaf_values = []
        for i in range(self.n):
            p = b.echos.get(i)
            leaf_values.append(p["value"] if p is not None and p["root_hash"] == h else None)
        value = decode_from_shards(leaf_values, self.n, h, self.variant)
        self.decode_attempts.append((b.proposer, h, value is not None))
        if value is not None:
            b.decided = True
            b.output = value
            self.outputs.append((b.proposer, value))

    def run(self, events):
        for ev in events:
            self.handle(ev)
        return self
