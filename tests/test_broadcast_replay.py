"""Batched Broadcast epoch: the replay driver
``hbbft_amd/broadcast.py`` must emit the FaultLog, errors, outgoing messages, decode attempts and
outputs that ``src/broadcast.rs`` emits message by message (``oracle/broadcast.py``).

* CPU: the oracle reproduces the reference's own test properties (``tests/broadcast.rs``: every
  good node outputs the proposed value, for sizes 1..5, 8, 13 under the silent, propose and random
  adversaries with random and first delivery; 32 equal spaces at N = 8);
* CPU: the replay's control flow over a stand-in engine built on the oracle;
* GPU: the replay over the HIP engine (``hbx_merkle_validate_d``, ``hbx_broadcast_decode_leaves_d``,
  ``hbx_rs_encode_d`` / ``hbx_merkle_build_d`` / ``hbx_merkle_proofs_d``), for both Merkle digests,
  and the leaf-sharing decode against the plain one.
"""
import numpy as np
import pytest

from bc_scenarios import OracleEngine, check_against_oracle, epoch_scenario, simulate
from hbbft_amd.broadcast import BroadcastReplay
from oracle import broadcast as ob
from oracle import rs_merkle as rm

SIZES = [1, 2, 3, 4, 5, 8, 13]
ADVERSARIES = [("silent", "random"), ("silent", "first"), ("propose", "random"), ("propose", "first"),
               ("random", "random")]


def _value(adv):
    return b"RandomFoo" if adv == "random" else b"Foo"


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("adv,sched", ADVERSARIES)
def test_oracle_reference_properties(n, adv, sched):
    """tests/broadcast.rs: all good nodes output exactly the proposed value."""
    value = _value(adv)
    received, nodes = simulate(n, adv, sched, value, seed=1000 * n + len(adv) + len(sched))
    for node in nodes.values():
        assert node.outputs == [(0, value)]
    if adv == "propose" and n >= 4:
        # the faulty proposer's Values are faults at every good node but the targets' own
        assert any(k == ob.RECEIVED_VALUE_FROM_NON_PROPOSER for node in nodes.values() for _, k in node.faults)


def test_oracle_equal_leaves_silent():
    """tests/broadcast.rs test_8_broadcast_equal_leaves_silent: 32 spaces at N = 8."""
    _, nodes = simulate(8, "silent", "random", b" " * 32, seed=8)
    assert all(node.outputs == [(0, b" " * 32)] for node in nodes.values())


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("adv,sched", ADVERSARIES)
def test_replay_logic_simulated(n, adv, sched):
    received, nodes = simulate(n, adv, sched, _value(adv), seed=1000 * n + len(adv) + len(sched))
    for i, events in received.items():
        res = BroadcastReplay(OracleEngine(), n, i).run(events)
        check_against_oracle(res, nodes[i], n)


@pytest.mark.parametrize("variant", ["sha256", "sha3"])
@pytest.mark.parametrize("n,me,seed", [(7, 6, 1), (10, 9, 2), (13, 5, 3)])
def test_replay_logic_epoch(n, me, seed, variant):
    events, _ = epoch_scenario(n, me, seed, variant)
    node = ob.BroadcastNode(n, me, variant).run(events)
    eng = OracleEngine(variant)
    res = BroadcastReplay(eng, n, me).run(events)
    check_against_oracle(res, node, n)
    # the scenario's fault paths all happened
    kinds = {k for _, k in node.faults}
    assert {ob.RECEIVED_VALUE_FROM_NON_PROPOSER, ob.INVALID_PROOF} <= kinds
    assert {e for _, e in node.errors} == {ob.UNKNOWN_SENDER, ob.NO_SUCH_BROADCAST_INSTANCE}
    att2 = [ok for p, _, ok in node.decode_attempts if p == 2]
    assert att2 and not att2[0] and att2[-1], "proposer 2: failed decodes, then the retry succeeds"
    assert not any(ok for p, _, ok in node.decode_attempts if p == 3), "proposer 3 never decodes"
    decided = {p for p, _ in node.outputs}
    assert decided == set(range(n)) - {3}
    # repeated failed attempts with the same Echo set are decoded once
    assert res.engine_decodes <= len(node.decode_attempts)


SHORT_CASES = [(10, 9, 5, 8), (13, 5, 6, 11)]  # (n, me, seed, proposer with 1-byte leaves)


@pytest.mark.parametrize("variant", ["sha256", "sha3"])
@pytest.mark.parametrize("n,me,seed,short", SHORT_CASES)
def test_replay_logic_short_leaves(n, me, seed, short, variant):
    """A proposer whose leaves are only the index byte: proofs validate, Echo and Ready go out, the
    decode yields nothing (glue_shards: < 4 bytes) and the node stays undecided -- no error."""
    events, _ = epoch_scenario(n, me, seed, variant, short_leaves=short)
    node = ob.BroadcastNode(n, me, variant).run(events)
    res = BroadcastReplay(OracleEngine(variant), n, me).run(events)
    check_against_oracle(res, node, n)
    assert any(p == short for p, _, _ in node.decode_attempts)
    assert short not in {p for p, _ in node.outputs}


# ---- GPU --------------------------------------------------------------------------------------
def _gpu_engine(ctx, variant):
    from hbbft_amd.broadcast import GpuBroadcastEngine
    from hbbft_amd.hbx import MERKLE_SHA3, MERKLE_SHA256

    return GpuBroadcastEngine(ctx, MERKLE_SHA3 if variant == "sha3" else MERKLE_SHA256)


@pytest.mark.gpu
@pytest.mark.parametrize("adv,sched", ADVERSARIES)
def test_gpu_replay_simulated(hbx_ctx, adv, sched):
    eng = _gpu_engine(hbx_ctx, "sha256")
    for n in SIZES:
        received, nodes = simulate(n, adv, sched, _value(adv), seed=1000 * n + len(adv) + len(sched))
        for i, events in received.items():
            res = BroadcastReplay(eng, n, i).run(events)
            check_against_oracle(res, nodes[i], n)
            assert res.outputs == [(0, _value(adv))]


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["sha256", "sha3"])
@pytest.mark.parametrize("n,me,seed", [(7, 6, 1), (10, 9, 2), (13, 5, 3), (40, 39, 4)])
def test_gpu_replay_epoch(hbx_ctx, n, me, seed, variant):
    events, _ = epoch_scenario(n, me, seed, variant)
    node = ob.BroadcastNode(n, me, variant).run(events)
    res = BroadcastReplay(_gpu_engine(hbx_ctx, variant), n, me).run(events)
    check_against_oracle(res, node, n)
    assert res.engine_decodes <= len(node.decode_attempts)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["sha256", "sha3"])
@pytest.mark.parametrize("n,me,seed,short", SHORT_CASES)
def test_gpu_replay_short_leaves(hbx_ctx, n, me, seed, short, variant):
    events, _ = epoch_scenario(n, me, seed, variant, short_leaves=short)
    node = ob.BroadcastNode(n, me, variant).run(events)
    res = BroadcastReplay(_gpu_engine(hbx_ctx, variant), n, me).run(events)
    check_against_oracle(res, node, n)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["sha256", "sha3"])
@pytest.mark.parametrize("n,L", [(4, 9), (13, 64), (128, 2052), (128, 23832)])
def test_gpu_decode_leaves_matches_decode(hbx_ctx, n, L, variant):
    """hbx_broadcast_decode_leaves_d (present digests handed in) == hbx_broadcast_decode_d, with
    erasure patterns: none, the last f, one too many, and a wrong root."""
    import torch

    from hbbft_amd.hbx import MERKLE_SHA3, MERKLE_SHA256

    hbx_ctx.set_merkle_digest(MERKLE_SHA3 if variant == "sha3" else MERKLE_SHA256)
    k, m = rm.coding_counts(n)
    f = rm.num_faulty(n)
    rng = np.random.default_rng(n * 7 + L)
    inst = 4
    full = np.zeros((inst, n, L), dtype=np.uint8)
    full[:, :k] = rng.integers(0, 256, size=(inst, k, L), dtype=np.uint8)
    d = torch.from_numpy(full).cuda()
    hbx_ctx.rs_encode_d(d, k, m)
    full = d.cpu().numpy()
    present = np.ones((inst, n), dtype=np.uint8)
    present[1, n - f:] = 0
    present[2, : m + 1] = 0
    present[3, :f] = 0
    roots, digests = np.zeros((inst, 32), np.uint8), np.zeros((inst, n, 32), np.uint8)
    for i in range(inst):
        leaves = [bytes([j]) + full[i, j].tobytes() for j in range(n)]
        roots[i] = np.frombuffer(rm.MerkleTree(leaves, variant).root_hash(), dtype=np.uint8)
        for j in range(n):
            digests[i, j] = np.frombuffer(rm.hash_leaf(leaves[j], variant), dtype=np.uint8)
    roots[3, 0] ^= 1
    work = full.copy()
    work[present == 0] = 0xA5
    outs = []
    for leaves_mode in (False, True):
        w = torch.from_numpy(work).cuda()
        out = torch.zeros((inst, k * L), dtype=torch.uint8, device="cuda")
        ln = torch.zeros(inst, dtype=torch.int64, device="cuda")
        st = torch.zeros(inst, dtype=torch.int32, device="cuda")
        args = (torch.from_numpy(present).cuda(),)
        if leaves_mode:
            hbx_ctx.broadcast_decode_leaves_d(w, args[0], torch.from_numpy(digests).cuda(), torch.from_numpy(roots).cuda(),
                                              k, m, out, ln, st)
        else:
            hbx_ctx.broadcast_decode_d(w, args[0], torch.from_numpy(roots).cuda(), k, m, out, ln, st)
        torch.cuda.synchronize()
        outs.append((st.cpu().numpy(), ln.cpu().numpy(), out.cpu().numpy(), w.cpu().numpy()))
    (s0, l0, o0, w0), (s1, l1, o1, w1) = outs
    np.testing.assert_array_equal(s0, s1)
    np.testing.assert_array_equal(l0, l1)
    np.testing.assert_array_equal(o0, o1)
    assert s1[0] == 0 and s1[1] == 0 and s1[2] == -9 and s1[3] == -10
    np.testing.assert_array_equal(w1[:2], full[:2])
