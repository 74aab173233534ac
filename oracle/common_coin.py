"""Common Coin, one message at a time -- TEST ORACLE ONLY.

Only ``tests/`` (and fixture scripts under ``tests/golden/``) may import this.  It restates what
``src/common_coin.rs`` does at ONE node for a set of coin instances (one per nonce: the
``CommonCoin`` each Agreement instance owns), line by line, with the CPU crypto of
``oracle/threshold.py``, so that the batched replay in ``hbbft_amd/common_coin.py`` (one engine
call for every signature share of the round) can be checked to emit the same FaultLog, errors,
messages and outputs, in the same order:

* ``input``            common_coin.rs:90-97 -- once: ``had_input``; ``get_coin`` (:138-147): a
  validator signs the nonce (``SecretKeyShare::sign``, :142), sends the share to all and handles
  it as its own message (``handle_share``) -- unless that returns an error, which drops the step
  and with it the message (``?`` at :145; the error is filed under ``None``); a non-validator goes
  straight to ``try_output``;
* ``handle_message``   :100-110 -- ignored once ``terminated`` (no fault even for a bad share);
* ``handle_share``     :149-161 -- unknown sender -> ``Err(UnknownSender)``; a share that does not
  verify (``PublicKeyShare::verify``, :151) -> fault ``UnverifiedSignatureShareSender`` and NO
  ``try_output``; otherwise insert (BTreeMap: a later share of the same sender replaces the
  earlier one) and ``try_output``;
* ``try_output``       :163-181 -- needs ``had_input`` and more than f shares; combines the shares
  held at that moment (``combine_signatures``: the first t = f + 1 in node order, :183-190) and
  checks the result against the master key (:191-204, ``Err(VerificationFailed)``, state kept, so
  a later share retries); on success outputs ``Signature::parity`` and terminates.

Message model: ``("input", inst)`` -- this node's input to instance ``inst``;
``("share", sender, inst, sig96)`` -- a ``CommonCoinMessage``.  ``sig96`` that is not a G2
subgroup point is rejected by serde before CommonCoin sees it (no fault, no state change); a
sender >= n is not a validator (``UnknownSender``).  Node indices are the BTreeMap order of the
node ids (messaging.rs:246-250).
"""
from __future__ import annotations

from . import bls12_381 as bls
from . import threshold as tc

UNVERIFIED_SIGNATURE_SHARE_SENDER = "UnverifiedSignatureShareSender"
UNKNOWN_SENDER = "UnknownSender"
VERIFICATION_FAILED = "VerificationFailed"
COMBINE_FAILED = "CombineAndVerifySigCrypto"


def decode_sig(b: bytes):
    """SignatureShare deserialisation (G2 into_affine: curve + subgroup); None if it fails."""
    try:
        return bls.g2_decompress(bytes(b))
    except ValueError:
        return None


class _Coin:
    __slots__ = ("nonce", "h", "received", "had_input", "terminated")

    def __init__(self, nonce: bytes, h):
        self.nonce = nonce
        self.h = h  # hash_g2(nonce), a pure function of the nonce (cached)
        self.received = {}  # sender -> share point (BTreeMap<N, SignatureShare>)
        self.had_input = False
        self.terminated = False


class CoinNode:
    """Node ``me`` (None: an observer, not a validator) of n validators, one CommonCoin per nonce."""

    def __init__(self, n: int, me, pk_set: tc.PublicKeySet, sk_share, nonces, variant: str = tc.DEFAULT_DIGEST):
        self.n = n
        self.f = (n - 1) // 3  # NetworkInfo::num_faulty, messaging.rs:258
        self.me = me
        self.pk_set = pk_set
        self.pk_shares = [pk_set.public_key_share(i) for i in range(n)]
        self.sk = sk_share
        self.variant = variant
        self.coins = [_Coin(bytes(x), tc.hash_g2(bytes(x), variant)) for x in nonces]
        self.faults = []  # (sender, FaultKind name), in emission order
        self.errors = []  # (sender, error name): handle_message returned Err (None: our input call)
        self.sent = []  # (inst, sig point): our share sent to all
        self.outputs = []  # (inst, parity) in output order
        self.combines = []  # (inst, senders combined, ok) as try_output ran them

    # -- crypto (one method per threshold_crypto call) --------------------------------------------
    def _verify(self, sender: int, share, coin: _Coin) -> bool:
        return tc.verify_sig(self.pk_shares[sender], share, coin.nonce, self.variant, hash_pt=coin.h)

    def _sign(self, coin: _Coin):
        return tc.sign(self.sk, coin.nonce, self.variant, hash_pt=coin.h)

    def _combine(self, shares):
        return tc.combine_signatures(self.pk_set, shares)

    def _master_verify(self, sig, coin: _Coin) -> bool:
        return tc.verify_sig(self.pk_set.public_key(), sig, coin.nonce, self.variant, hash_pt=coin.h)

    # -- handlers ---------------------------------------------------------------------------------
    def handle(self, event):
        if event[0] == "input":
            self._input(event[1])
        elif event[0] == "share":
            _, sender, inst, sig96 = event
            sig = decode_sig(sig96)
            if sig is None:
                return  # never reaches CommonCoin
            coin = self.coins[inst]
            if coin.terminated:
                return  # handle_message: ignored after termination (:105-110)
            self._handle_share(inst, sender, sig)
        else:
            raise ValueError(event[0])

    def _input(self, inst: int):
        coin = self.coins[inst]
        if coin.had_input:
            return
        coin.had_input = True
        if self.me is None:  # not a validator (:139-141)
            self._try_output(inst, None)
            return
        share = self._sign(coin)
        # get_coin (:142-146) builds the Target::All message, then `step.extend(self.handle_share(..)?)`:
        # an Err from our own share's try_output drops the whole step, message included -- the share
        # is never sent, and had_input stays set, so it never will be
        n_err = len(self.errors)
        self._handle_share(inst, self.me, share, who=None)
        if len(self.errors) == n_err:
            self.sent.append((inst, share))

    def _handle_share(self, inst: int, sender: int, share, who=-1):
        """``who``: whose call returns an error (-1: the message's sender; None: our own input)."""
        who = sender if who == -1 else who
        coin = self.coins[inst]
        if not 0 <= sender < self.n:
            self.errors.append((who, UNKNOWN_SENDER))
            return
        if not self._verify(sender, share, coin):
            self.faults.append((sender, UNVERIFIED_SIGNATURE_SHARE_SENDER))
            return
        coin.received[sender] = share
        self._try_output(inst, who)

    def _try_output(self, inst: int, who):
        """``who``: the sender of the message being handled (None: our own input), whose
        handle_message / input call returns the error."""
        coin = self.coins[inst]
        if not (coin.had_input and len(coin.received) > self.f):
            return
        senders = sorted(coin.received)
        try:
            sig = self._combine([(i, coin.received[i]) for i in senders])
        except (tc.NotEnoughShares, tc.DuplicateEntry):
            self.combines.append((inst, tuple(senders), False))
            self.errors.append((who, COMBINE_FAILED))
            return
        if not self._master_verify(sig, coin):
            self.combines.append((inst, tuple(senders), False))
            self.errors.append((who, VERIFICATION_FAILED))
            return
        self.combines.append((inst, tuple(senders), True))
        coin.terminated = True
        self.outputs.append((inst, tc.parity(sig)))

    def run(self, events):
        for ev in events:
            self.handle(ev)
        return self
