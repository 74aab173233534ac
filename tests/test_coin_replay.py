"""Batched Common Coin round: ``hbbft_amd/common_coin.py`` (CoinReplay: one
verification pass over every signature share, the reference's control flow replayed, the combine
restricted to the shares held at trigger time) must emit the FaultLog, errors, messages, combine
attempts and outputs that ``src/common_coin.rs`` emits message by message
(``oracle/common_coin.py``).

* CPU: the replay over a stand-in engine built on the oracle, node and observer, several sizes;
  a combination the engine reports as failing (VerificationFailed) is retried where the reference
  retries;
* GPU: the replay over the HIP engine (``hbx_verify_sig_shares_d``, ``hbx_combine_signatures_d``),
  and the device API against the host API on a coin fixture.
"""
import numpy as np
import pytest

from coin_scenarios import OracleCoinEngine, check_against_oracle, coin_scenario
from hbbft_amd.common_coin import CoinReplay
from oracle import common_coin as oc

CASES = [(4, 3, 4, 1), (4, None, 4, 2), (7, 6, 5, 3), (10, 2, 4, 4)]


def _oracle(n, me, ns, sks, pks, events):
    sk = None if me is None else sks.secret_key_share(me)
    return oc.CoinNode(n, me, pks, sk, ns).run(events)


@pytest.mark.parametrize("n,me,count,seed", CASES)
def test_replay_logic(n, me, count, seed):
    ns, sks, pks, events = coin_scenario(n, me, count, seed)
    node = _oracle(n, me, ns, sks, pks, events)
    eng = OracleCoinEngine(pks, None if me is None else sks.secret_key_share(me))
    res = CoinReplay(eng, n, me).run(ns, events)
    check_against_oracle(res, node)
    # the scenario's paths all happened
    assert {k for _, k in node.faults} == {oc.UNVERIFIED_SIGNATURE_SHARE_SENDER}
    assert [e for e in node.errors] == [(n + 2, oc.UNKNOWN_SENDER)]
    done = {i for i, _ in node.outputs}
    assert 0 in done and 1 in done and 2 not in done
    assert res.engine_combines == 1


class _FlakyCombine(OracleCoinEngine):
    """The first combination of instance 0 fails the master check (as a wrong share set would):
    the reference keeps the instance open, logs VerificationFailed and retries on the next share."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.calls = 0

    def combine(self, use, t):
        st, ok, par = super().combine(use, t)
        self.calls += 1
        if self.calls == 1:
            ok[0] = False
        return st, ok, par


def test_replay_retries_a_failed_combination():
    n, me, count, seed = 4, 3, 4, 5
    ns, sks, pks, events = coin_scenario(n, me, count, seed)
    eng = _FlakyCombine(pks, sks.secret_key_share(me))
    res = CoinReplay(eng, n, me).run(ns, events)

    class Node(oc.CoinNode):
        first = True

        def _master_verify(self, sig, coin):
            if coin is self.coins[0] and Node.first:
                Node.first = False
                return False
            return super()._master_verify(sig, coin)

    node = Node(n, me, pks, sks.secret_key_share(me), ns).run(events)
    check_against_oracle(res, node)
    # instance 0's threshold is crossed by our own share at input time: the failed combination is
    # our input call's error, and get_coin's `?` (common_coin.rs:145) drops the step with our
    # outgoing share -- it is never sent (had_input stays set)
    assert (None, oc.VERIFICATION_FAILED) in node.errors
    assert 0 not in {inst for inst, _ in node.sent}
    assert 0 not in {inst for inst, _ in res.sent}
    assert {inst for inst, _ in node.sent} == {inst for inst, _ in res.sent} != set()
    assert 0 in {inst for inst, _ in node.outputs}  # retried on the next share, then output
    assert res.engine_combines == 2


# ---- GPU --------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("n,me,count,seed", CASES)
def test_gpu_replay(hbx_ctx, n, me, count, seed):
    from oracle import bls12_381 as bls

    ns, sks, pks, events = coin_scenario(n, me, count, seed)
    node = _oracle(n, me, ns, sks, pks, events)
    hbx_ctx.set_pk_shares([bls.g1_compress(pks.public_key_share(i)) for i in range(n)])
    from hbbft_amd.common_coin import GpuCoinEngine

    sk32 = None if me is None else sks.secret_key_share(me).to_bytes(32, "big")
    eng = GpuCoinEngine(hbx_ctx, bls.g1_compress(pks.public_key()), sk32)
    for lanes in (0, 1):
        hbx_ctx.set_verify_lanes(lanes)
        res = CoinReplay(eng, n, me).run(ns, events)
        check_against_oracle(res, node)
        assert hbx_ctx.coin_lanes_used() == (2 if lanes == 0 else 1)
    hbx_ctx.set_verify_lanes(0)
