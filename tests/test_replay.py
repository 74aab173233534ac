"""HoneyBadger epoch replay: the batched driver hbbft_amd/honey_badger.py must
emit the FaultLog, errors and Batch that honey_badger.rs emits message by message.

* test_oracle_restatement_reproduces_fixture -- the fixture's expectations are what the
  message-at-a-time restatement (oracle/honey_badger.py) produces for its events;
* test_replay_logic_with_oracle_statuses -- the batched replay, fed the oracle's per-message
  verification results through a stand-in engine (CPU), emits exactly those expectations;
* test_gpu_replay_matches_fixture -- the same replay over the real HIP engine (GPU).
"""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

from make_replay import ERROR_CODES, FAULT_CODES, NO_STATUS, load_events  # noqa: E402

from hbbft_amd.honey_badger import EpochReplay  # noqa: E402

FAULT_NAMES = {v: k for k, v in FAULT_CODES.items()}
ERROR_NAMES = {v: k for k, v in ERROR_CODES.items()}


def _load(tag):
    return dict(np.load(os.path.join(HERE, "golden", f"hb_replay_{tag}.npz"), allow_pickle=False))


def _expect(d):
    faults = [(int(a), FAULT_NAMES[int(b)]) for a, b in zip(d["expect_fault_node"], d["expect_fault_kind"])]
    errors = [(int(a), ERROR_NAMES[int(b)]) for a, b in zip(d["expect_error_node"], d["expect_error_kind"])]
    batch = None
    if bool(d["expect_batch"]):
        off = d["expect_batch_off"]
        batch = {int(j): d["expect_batch_blob"][int(off[q]):int(off[q + 1])].tobytes()
                 for q, j in enumerate(d["expect_batch_proposers"])}
    return faults, errors, batch


def _check(res, d):
    faults, errors, batch = _expect(d)
    assert res.faults == faults
    assert res.errors == errors
    assert res.batch == batch


class OracleStatusEngine:
    """Stands in for hbx.Context with the oracle's per-message verification results."""

    def __init__(self, d, events):
        self.acs = [int(j) for j in d["acs_proposers"]]
        self.col = {j: q for q, j in enumerate(self.acs)}
        self.ct = d["expect_ct_status"]
        self.by_msg = {}
        for k, ev in enumerate(events):
            st = int(d["expect_ev_status"][k])
            if ev[0] == "share" and st != NO_STATUS:
                self.by_msg[(self.col[ev[2]], ev[1], ev[3])] = st
        self.last = None
        self.plain = {}
        _, _, batch = _expect(d)
        self.plain = batch or {}

    def set_own_share(self, me, sk):
        self.me = me

    def prepare_ciphertexts(self, cts):
        assert len(cts) == len(self.acs)
        return self.ct == 1

    def ct_status(self, p):
        return self.ct.copy()

    def verify_dec_shares(self, shares, present):
        p, n, _ = shares.shape
        st = np.full((p, n), 2, dtype=np.uint8)  # absent
        for j in range(p):
            for i in range(n):
                if present[j, i]:
                    st[j, i] = self.by_msg[(j, i, shares[j, i].tobytes())]
        self.last = st
        return st == 1

    def share_status(self, p, n):
        return self.last

    def combine_decrypt(self, t):
        plains = [self.plain.get(j) for j in self.acs]
        return plains, np.array([0 if x is not None else -3 for x in plains], dtype=np.int32)


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_oracle_restatement_reproduces_fixture(tag):
    from oracle import honey_badger as ohb
    from oracle import threshold as tc
    from make_replay import keys

    d = _load(tag)
    sks, pks = keys()
    node = ohb.EpochNode(int(d["n"]), int(d["me"]), pks, sks.secret_key_share(int(d["me"]))).run(load_events(d))
    faults, errors, batch = _expect(d)
    assert node.faults == faults and node.errors == errors and node.batch == batch
    assert tc.DEFAULT_DIGEST == "sha256"


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_replay_logic_with_oracle_statuses(tag):
    d = _load(tag)
    events = load_events(d)
    eng = OracleStatusEngine(d, events)
    res = EpochReplay(eng, int(d["n"]), int(d["me"]), d["sk_me"].tobytes()).run(events)
    _check(res, d)


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_gpu_replay_matches_fixture(hbx_ctx, tag):
    d = _load(tag)
    assert (hbx_ctx.set_pk_shares([row.tobytes() for row in d["pk_comp"]]) == 0).all()
    events = load_events(d)
    try:
        res = EpochReplay(hbx_ctx, int(d["n"]), int(d["me"]), d["sk_me"].tobytes()).run(events)
    finally:
        hbx_ctx.set_own_share(0, None)
    # the engine's statuses are the oracle's, message by message
    for k, st in enumerate(res.share_status):
        want = int(d["expect_ev_status"][k])
        if want != NO_STATUS:
            assert st == want, f"event {k}"
    assert [res.ct_status[int(j)] for j in d["acs_proposers"]] == d["expect_ct_status"].tolist()
    _check(res, d)
