"""The reference's own test properties, run as seeded GPU tests through the engine (VERDICT r2
item 7).  The Broadcast ones (tests/broadcast.rs) are in test_broadcast_replay.py.

* Common Coin (``tests/common_coin.rs:54-73, 79-133``): for the reference's network sizes (1, then
  growing by 3..6) and 200 / 50 nonces ``"My very unique nonce {id:x}:{i}"``, the f faulty nodes
  silent, every good node -- each combining a different set of at least f + 1 signature shares, as
  arrival order would give it -- must output the same coin, equal to the parity of the master
  signature (oracle ``threshold.sign`` with the master key), and the coin sides must pass the
  reference's ``check_coin_distribution``.
* HoneyBadger (``tests/honey_badger.rs:99-130, 192-245``): sizes {1, 2, 3, 5, 7}, the f faulty
  nodes running the FaultyShareAdversary (a share of a ciphertext of "X marks the spot" to every
  proposer), random and first delivery: every good node's decryption sub-path, replayed by
  ``EpochReplay`` on the GPU, must output the batch of every good proposer's contribution, and its
  FaultLog must equal the message-at-a-time oracle's (``oracle/honey_badger.py``) with known
  answers standing in for its pairings (the adversary's shares are wrong by construction).
"""
import math
import random

import numpy as np
import pytest

from oracle import honey_badger as ohb
from oracle import threshold as tc
from oracle import bls12_381 as bls


# ---- Common Coin -------------------------------------------------------------------------------
GOOD_SAMPLE_SET = 400.0


def check_coin_distribution(num_samples: int, count_true: int, count_false: int):
    """tests/common_coin.rs:56-73."""
    expected_share = 0.4
    max_gain = math.log2(GOOD_SAMPLE_SET)
    gain = min(math.log2(num_samples), max_gain)
    step = expected_share / max_gain
    min_throws = int(num_samples * gain * step)
    assert count_true > min_throws, (count_true, min_throws)
    assert count_false > min_throws, (count_false, min_throws)


def coin_sizes(num_samples: int, rng: random.Random):
    """tests/common_coin.rs:85-93: 1, then log2(400) - log2(samples) sizes growing by 3..6."""
    sizes = [1]
    for _ in range(int(math.log2(GOOD_SAMPLE_SET) - math.log2(num_samples))):
        sizes.append(sizes[-1] + rng.randrange(3, 7))
    return sizes


@pytest.mark.gpu
@pytest.mark.parametrize("num_samples", [200, 50])
def test_gpu_common_coin_distribution(hbx_ctx, num_samples):
    from hbbft_amd import netinfo

    rng = random.Random(num_samples)
    for size in coin_sizes(num_samples, rng):
        f = (size - 1) // 3
        good = size - f
        sks, sk_shares, master_sk = netinfo.generate_keys(size, seed=0x636F696E + size)
        t = sks.threshold + 1
        pk = hbx_ctx.public_keys(sk_shares)
        master_pk = hbx_ctx.public_keys(master_sk)[0].tobytes()
        assert (hbx_ctx.set_pk_shares([r.tobytes() for r in pk]) == 0).all()
        uid = rng.getrandbits(64)
        nonces = [f"My very unique nonce {uid:x}:{i}".encode() for i in range(num_samples)]
        hbx_ctx.prepare_nonces(nonces)
        sigs = hbx_ctx.sign(sk_shares)
        coins = None
        for node in range(good):
            # the shares this good node combines: its own plus a random >= f other good nodes'
            present = np.zeros((num_samples, size), dtype=bool)
            for s in range(num_samples):
                others = [i for i in range(good) if i != node]
                pick = rng.sample(others, rng.randint(min(f, len(others)), len(others)))
                present[s, [node] + pick] = True
            valid = hbx_ctx.verify_sig_shares(sigs, present)
            assert (valid == present).all()
            sig, st, ok, par = hbx_ctx.combine_signatures(master_pk, t)
            assert (st == 0).all() and ok.all()
            if coins is None:
                coins, sig0 = par.copy(), sig.copy()
            else:
                assert (par == coins).all() and (sig == sig0).all(), "good nodes disagree on the coin"
        master = int.from_bytes(master_sk[0].tobytes(), "big")
        for s in range(0, num_samples, max(1, num_samples // 25)):
            want = tc.sign(master, nonces[s])
            assert bls.g2_compress(want) == sig0[s].tobytes()
            assert tc.parity(want) == bool(coins[s])
        check_coin_distribution(num_samples, int(coins.sum()), int((~coins).sum()))


# ---- HoneyBadger with the FaultyShareAdversary ---------------------------------------------------
class _NoKeys:
    def public_key_share(self, i):
        return None


class KnownAnswerEpochNode(ohb.EpochNode):
    """oracle/honey_badger.py's control flow with known answers for its threshold_crypto calls:
    a share verifies iff it is the sender's honest share of that proposer's ciphertext."""

    def __init__(self, n, me, honest, contributions, ct_owner):
        super().__init__(n, me, _NoKeys(), None)
        self.honest = honest  # (proposer, sender) -> share48
        self.contributions = contributions
        self.ct_owner = ct_owner  # ciphertext bytes -> proposer

    def _decode_share(self, share48):
        return ("ok", bytes(share48))

    def _decode_ciphertext(self, ct):
        return tuple(bytes(x) for x in ct)

    def _ciphertext_verify(self, proposer, ct):
        return True

    def _verify_share(self, sender, share, proposer, ct):
        return sender < self.n and self.honest.get((proposer, sender)) == share

    def _own_share(self, ct):
        return self.honest[(self.ct_owner[ct], self.me)]

    def _decrypt(self, shares, ct):
        return self.contributions[self.ct_owner[ct]]


def hb_network(ctx, n: int, seed: int):
    """Keys, the good proposers' ciphertexts and every share of a network of n nodes (f faulty)."""
    from hbbft_amd import netinfo

    f = (n - 1) // 3
    good = n - f
    sks, sk_shares, master_sk = netinfo.generate_keys(n, seed=0x68620000 + seed)
    pk = ctx.public_keys(sk_shares)
    master_pk = ctx.public_keys(master_sk)[0].tobytes()
    rng = np.random.default_rng(seed)
    contributions = {p: rng.integers(0, 256, size=int(rng.integers(1, 200)), dtype=np.uint8).tobytes()
                     for p in range(good)}
    props = list(range(good))
    r = netinfo.scalars_to_be32(netinfo.random_scalars(rng, good + 1))
    cts = ctx.encrypt(master_pk, [contributions[p] for p in props] + [b"X marks the spot"], r)
    u48 = np.stack([np.frombuffer(c[0], dtype=np.uint8) for c in cts])
    shares = ctx.decrypt_shares(sk_shares, u48)  # (good + 1, n, 48); the last row: the fake ciphertext
    return dict(f=f, good=good, sk_shares=sk_shares, pk=pk, t=sks.threshold + 1, contributions=contributions,
                cts={p: cts[p] for p in props}, shares=shares)


def node_events(net, n: int, me: int, scheduler: str, rng: random.Random):
    """What good node `me` receives: every other node's DecryptionShare for every proposer (the f
    faulty nodes send their share of the fake ciphertext, to every proposer id 0..n-1) and the
    CommonSubset output, in random or first-come order."""
    good, f = net["good"], net["f"]
    msgs = []
    for s in range(n):
        if s == me:
            continue
        if s < good:
            msgs += [("share", s, p, net["shares"][p, s].tobytes()) for p in range(good)]
        else:
            msgs += [("share", s, p, net["shares"][good, s].tobytes()) for p in range(n)]
    acs = ("acs", {p: net["cts"][p] for p in range(good)})
    if scheduler == "random":
        rng.shuffle(msgs)
        msgs.insert(rng.randrange(len(msgs) + 1), acs)
    else:  # "first": the shares in sender order, the CommonSubset output in the middle
        msgs.insert(len(msgs) // 2, acs)
    return msgs


@pytest.mark.gpu
@pytest.mark.parametrize("scheduler", ["random", "first"])
def test_gpu_honey_badger_faulty_share(hbx_ctx, scheduler):
    from hbbft_amd.honey_badger import EpochReplay

    for n in (1, 2, 3, 5, 7):
        net = hb_network(hbx_ctx, n, seed=n)
        assert (hbx_ctx.set_pk_shares([r.tobytes() for r in net["pk"]]) == 0).all()
        good = net["good"]
        honest = {(p, s): net["shares"][p, s].tobytes() for p in range(good) for s in range(n)}
        owner = {tuple(bytes(x) for x in net["cts"][p]): p for p in range(good)}
        rng = random.Random(1000 + n)
        for me in range(good):
            events = node_events(net, n, me, scheduler, rng)
            res = EpochReplay(hbx_ctx, n, me, net["sk_shares"][me].tobytes()).run(events)
            want = KnownAnswerEpochNode(n, me, honest, net["contributions"], owner).run(events)
            assert res.batch == net["contributions"], (n, me)  # the reference's property
            assert res.batch == want.batch
            assert res.faults == want.faults, (n, me)
            assert res.errors == want.errors
            bad = set(range(good, n))
            assert {s for s, _ in res.faults} <= bad
