"""Message logs for the Broadcast replay tests (row f3): what one node receives in an epoch.

* ``simulate`` -- the reference's own test shape (``tests/broadcast.rs``): a network of good nodes
  and f faulty ones runs ONE Broadcast instance (proposer 0) with the message-at-a-time oracle
  (``oracle/broadcast.py``) at every good node, messages delivered by a seeded scheduler ("random"
  or "first", ``MessageScheduler``), with the reference's adversaries: ``silent``
  (``SilentAdversary``), ``propose`` (``ProposeAdversary``: the first faulty node proposes
  b"Fake news" for the same instance) and ``random`` (``RandomAdversary(0.2, 0.2)``: Values
  addressed to a faulty node are re-sent by it to a random node, and faulty nodes inject random
  messages -- at most 8 each, so that the run ends).  Returns each good node's received events in
  order, and its oracle node.
* ``epoch_scenario`` -- every instance of an epoch at once at one node, with the fault paths of
  broadcast.rs:407-551 placed on purpose: a Value from a non-proposer, an invalid Value proof, a
  duplicate Echo, an Echo with a corrupted sibling, Echos and Readys for a second root (an
  equivocating proposer), a decode that fails (a missing shard reconstructed from a tampered
  one) and is retried when the last Echo arrives, leaves of different lengths (never decodes),
  Readys repeated / for unknown roots, an unknown sender and an unknown instance.
"""
from __future__ import annotations

import random

import numpy as np

from oracle import broadcast as ob
from oracle import rs_merkle as rm


def _junk_proof(rng: random.Random, n: int):
    depth = rng.randint(0, 4)
    lemma = [(rng.randbytes(32), (rng.choice("LR"), rng.randbytes(32))) for _ in range(depth)]
    lemma.append((rng.randbytes(32), None))
    return {"root_hash": rng.randbytes(32), "lemma": lemma, "value": bytes([rng.randrange(n)]) + rng.randbytes(rng.randint(0, 9))}


def simulate(n: int, adversary: str, scheduler: str, value: bytes, seed: int, variant: str = "sha256",
             max_steps: int = 200000):
    f = (n - 1) // 3
    good = list(range(n - f))
    bad = list(range(n - f, n))
    rng = random.Random(seed)
    nodes = {i: ob.BroadcastNode(n, i, variant) for i in good}
    received = {i: [] for i in good}
    queue = []  # (target, event)

    def flush(i):
        node = nodes[i]
        for target, ev in node.outbox:
            dests = [target] if target is not None else [j for j in range(n) if j != i]
            for d in dests:
                queue.append((d, ev))
        node.outbox.clear()

    def deliver(d, ev):
        if d in nodes:
            received[d].append(ev)
            nodes[d].handle(ev)
            flush(d)
        elif adversary == "random" and ev[0] == "value" and rng.random() < 0.2:
            # RandomAdversary::push_message: a Value addressed to a faulty node is re-sent by it
            queue.append((rng.randrange(n), ("value", d, ev[2], ev[3])))

    received[0].append(("input", value))
    nodes[0].handle(("input", value))
    flush(0)
    if adversary == "propose" and bad:
        # ProposeAdversary: the first faulty node runs Broadcast::input(b"Fake news") for the same
        # instance; its Value and Echo messages go out under its own id
        adv = bad[0]
        _, leaves, tree = rm.send_shards(b"Fake news", n, variant)
        for i, leaf in enumerate(leaves):
            p = tree.gen_proof(leaf)
            if i != adv:
                queue.append((i, ("value", adv, 0, p)))
            else:
                for j in range(n):
                    if j != adv:
                        queue.append((j, ("echo", adv, 0, p)))
    steps = injected = 0
    while queue and not all(nodes[i].inst[0].decided for i in good):
        steps += 1
        assert steps < max_steps, "simulation did not terminate"
        if adversary == "random" and bad and injected < 8 * len(bad) and rng.random() < 0.2:
            injected += 1
            src = rng.choice(bad)
            kind = rng.choice(["value", "echo", "ready"])
            payload = rng.randbytes(32) if kind == "ready" else _junk_proof(rng, n)
            for j in range(n):
                if j != src:
                    queue.append((j, (kind, src, 0, payload)))
        k = rng.randrange(len(queue)) if scheduler == "random" else 0
        d, ev = queue.pop(k)
        deliver(d, ev)
    return received, nodes


def _tree(shards, variant):
    leaves = [bytes([i & 0xFF]) + bytes(s) for i, s in enumerate(shards)]
    return leaves, rm.MerkleTree(leaves, variant)


def epoch_scenario(n: int, me: int, seed: int, variant: str = "sha256", short_leaves: int = None):
    """One node's receive log for all n instances of an epoch (n >= 7).  ``short_leaves``: that
    proposer (>= 7) sends a valid tree whose leaves are only the index byte (a Byzantine proposal
    every state machine accepts; its decode glues fewer than 4 bytes and yields nothing)."""
    assert n >= 7
    rng = random.Random(seed)
    f = (n - 1) // 3
    k, m = rm.coding_counts(n)
    values = [bytes(rng.randbytes(rng.randint(1, 3000))) for _ in range(n)]
    values[1] = values[0][:len(values[0])]  # two proposers with equal sizes (one decode group)
    trees = {}
    for p in range(n):
        _, leaves, tree = rm.send_shards(values[p], n, variant)
        trees[p] = (leaves, tree)
    # proposer 2 tampers with data shard 0 after encoding: only a decode with all N Echos present
    # (no reconstruction) reproduces its root -- the first decode fails, the retry succeeds
    shards2 = rm.send_shards(values[2], n, variant)[0].copy()
    shards2[0, 5 % shards2.shape[1]] ^= 0x5A
    trees[2] = _tree(shards2, variant)
    # proposer 3: leaves of two lengths (rse IncorrectShardSize: never decodes)
    sh3 = [bytes(s) for s in rm.send_shards(values[3], n, variant)[0]]
    sh3[1] = sh3[1] + b"\x00"
    trees[3] = _tree(sh3, variant)
    if short_leaves is not None:
        assert 7 <= short_leaves < n and short_leaves != me
        trees[short_leaves] = _tree([b""] * n, variant)
    # proposer 4 equivocates: a second tree (another value) for the nodes >= n - f
    _, leaves4b, tree4b = rm.send_shards(b"equivocation" * 7, n, variant)

    events = []
    per_inst = []
    for p in range(n):
        leaves, tree = trees[p]
        ev = []
        if p == me:
            ev.append(("input", values[p]))
        else:
            ev.append(("value", p, p, tree.gen_proof(leaves[me])))
        senders = [i for i in range(n) if i != me]
        rng.shuffle(senders)
        if p == 2:
            # all Readys first, then the Echos (sender 0's, the tampered shard, early), the shard of
            # the last sender arriving last: decodes with shards missing fail until it is in
            senders.remove(0)
            senders = [0] + senders
            for i in range(n):
                if i != me:
                    ev.append(("ready", i, p, tree.root_hash()))
        for i in senders:
            if p == 4 and i >= n - f:
                ev.append(("echo", i, p, tree4b.gen_proof(leaves4b[i])))
            else:
                ev.append(("echo", i, p, tree.gen_proof(leaves[i])))
        if p != 2:
            for i in range(n):
                if i != me:
                    h = tree4b.root_hash() if (p == 4 and i >= n - f) else tree.root_hash()
                    ev.append(("ready", i, p, h))
        per_inst.append(ev)
    # interleave the instances: a random merge keeping each instance's order
    cursors = [0] * n
    while any(cursors[p] < len(per_inst[p]) for p in range(n)):
        p = rng.choice([q for q in range(n) if cursors[q] < len(per_inst[q])])
        events.append(per_inst[p][cursors[p]])
        cursors[p] += 1
    # faults sprinkled in
    extra = []
    leaves5, tree5 = trees[5]
    other = (me + 1) % n
    extra.append(("value", other, 5, tree5.gen_proof(leaves5[me])))  # ReceivedValueFromNonProposer
    bad = dict(tree5.gen_proof(leaves5[me]))
    bad["value"] = bad["value"][:-1] + bytes([bad["value"][-1] ^ 1])
    extra.append(("value", 6, 6, dict(bad)))  # invalid Value proof (value of another instance)
    extra.append(("echo", other, 5, tree5.gen_proof(leaves5[other])))  # duplicate Echo (ignored)
    p6 = trees[6][1].gen_proof(trees[6][0][other])
    lem = list(p6["lemma"])
    if len(lem) > 1:
        h, (side, sib) = lem[0]
        lem[0] = (h, (side, bytes([sib[0] ^ 0x80]) + sib[1:]))
    extra.append(("echo", other, 6, dict(p6, lemma=lem)))  # corrupted sibling
    extra.append(("echo", other, 0, trees[0][1].gen_proof(trees[0][0][(other + 1) % n])))  # wrong position
    extra.append(("ready", other, 5, trees[5][1].root_hash()))  # repeated Ready
    extra.append(("ready", (other + 2) % n, 0, b"\x77" * 32))  # Ready for an unknown root
    extra.append(("echo", n + 3, 0, trees[0][1].gen_proof(trees[0][0][0])))  # unknown sender
    extra.append(("ready", 1, n + 1, trees[0][1].root_hash()))  # no such instance
    extra.append(("echo", other, 1, {"root_hash": b"\x01" * 32, "lemma": [], "value": b""}))  # malformed
    # the invalid Value and the corrupted-sibling Echo come first (before the real ones, which would
    # make them ignored duplicates); the rest anywhere
    events = extra[1:2] + extra[3:4] + events
    for ev in extra[:1] + extra[2:3] + extra[4:]:
        events.insert(rng.randrange(len(events) + 1), ev)
    return events, values


def proofs_equal(a, b) -> bool:
    return (bytes(a["root_hash"]) == bytes(b["root_hash"]) and bytes(a["value"]) == bytes(b["value"])
            and [(bytes(h), None if s is None else (s[0], bytes(s[1]))) for h, s in a["lemma"]]
            == [(bytes(h), None if s is None else (s[0], bytes(s[1]))) for h, s in b["lemma"]])


def check_against_oracle(res, node, n):
    """A BroadcastReplay result equals the oracle node's record."""
    assert res.faults == node.faults
    assert res.errors == node.errors
    assert res.sent == node.sent
    assert res.outputs == node.outputs
    assert res.decode_attempts == node.decode_attempts
    assert sorted(res.value_proofs) == sorted(node.value_proofs)
    for i, p in node.value_proofs.items():
        assert proofs_equal(res.value_proofs[i], p)


class OracleEngine:
    """A CPU stand-in for GpuBroadcastEngine built on the oracle (tests only): lets the replay's
    control flow be tested without a GPU."""

    def __init__(self, variant="sha256"):
        self.variant = variant
        self.decodes = 0

    def send_shards(self, value, n):
        _, leaves, tree = rm.send_shards(bytes(value), n, self.variant)
        return [tree.gen_proof(leaf) for leaf in leaves]

    def validate(self, proofs, nodes, n):
        return np.array([rm.validate_broadcast_proof(p, i, n, self.variant) for p, i in zip(proofs, nodes)], dtype=bool)

    def decode(self, attempts, n):
        self.decodes += len(attempts)
        out = []
        for vals, digests, root in attempts:
            for v, d in zip(vals, digests):
                if v is not None:
                    assert rm.hash_leaf(v, self.variant) == d  # the shared digests are the values' own
            out.append(ob.decode_from_shards(vals, n, root, self.variant))
        return out
