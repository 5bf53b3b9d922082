"""The Verify actor — the Python mirror of ``withVerifyActor`` in
haskell/Haskoin/Node/Verify.hs, policy for policy.

The node hands the actor the blocks and txs its peers send
(``PeerEvent (PeerMessage _ (MBlock b))`` / ``(MTx t)``, which
``Haskoin.Node.peerEvents`` drops at /root/reference/src/Haskoin/Node.hs:172);
the actor idiom is ``withChain`` (/root/reference/src/Haskoin/Node/Chain.hs:277-307):
a mailbox drained by one loop.

* **Batching.** A block is one ``verify_std_inputs`` call. Mempool txs are
  coalesced: the loop takes the first tx, then drains the mailbox until the
  batch holds ``max_inputs`` inputs (16,384 by default: the pair kernel's
  range) or ``max_wait_s`` has passed since the first tx, and
  makes ONE call for the whole batch (tx k of the batch is tx index k of the
  call). A message that does not fit (a block, or a tx past the bound) is held
  over and handled next, so the mailbox order is kept.
* **Errors.** A failed call (``HkvError``: HKV_E_INTERNAL when the call's
  multisig tail gave up, a device error) is re-submitted to the GPU up to
  ``retries`` times, then handed to ``fallback`` — in the Haskell actor,
  haskoin-core's own per-input ``verifyStdInput``, the CPU path the drop-in
  replaces; this package has no CPU verifier of its own, so the caller
  supplies it. With no fallback, or a fallback that raises, the batch's
  messages get ``VerifyFailed``. Nothing is raised into the loop: a verify
  failure never stops the actor (the Haskell actor runs under ``link``). A
  bug in the loop itself (e.g. ``publish`` raising) ends it; ``stop`` re-raises
  it and later posts raise at once instead of queueing unanswered.
"""
from __future__ import annotations

import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, List, Optional, Sequence, Tuple

from .lib import HkvError
from .sighash import verify_std_inputs

# Outcomes published per message (VerifyEvent in the Haskell module).


@dataclass(frozen=True)
class BlockVerified:
    key: Any


@dataclass(frozen=True)
class BlockRejected:
    key: Any
    bad: Tuple[Tuple[int, int], ...]  # (tx index, input index) of each failing input


@dataclass(frozen=True)
class TxVerified:
    key: Any


@dataclass(frozen=True)
class TxRejected:
    key: Any
    bad: Tuple[int, ...]  # input indices that fail verifyStdInput


@dataclass(frozen=True)
class VerifyFailed:
    key: Any
    error: str  # the GPU call failed after every retry and no fallback was given


@dataclass
class _Tx:
    key: Any
    tx: bytes
    inputs: Sequence[Tuple[int, bytes, int]]  # (input index, prevout scriptPubKey, prevout value)


@dataclass
class _Block:
    key: Any
    txs: Sequence[bytes]
    inputs: Sequence[Tuple[int, int, bytes, int]]  # (tx index, input index, prevout scriptPubKey, value)


_STOP = object()

Fallback = Callable[[Sequence[bytes], Sequence[Tuple[int, int, bytes, int]], Optional[int]], Sequence[bool]]


@dataclass
class VerifyActorConfig:
    """VerifyConfig of the Haskell module (net -> forkid)."""
    forkid: Optional[int] = None
    max_inputs: int = 16384
    max_wait_s: float = 0.002
    retries: int = 1
    fallback: Optional[Fallback] = None


@dataclass
class ActorStats:
    gpu_calls: int = 0          # verify_std_inputs calls, retries included
    gpu_failures: int = 0       # of which raised HkvError
    fallback_calls: int = 0
    batch_inputs: List[int] = field(default_factory=list)  # inputs per successful batch, in order
    errors: List[str] = field(default_factory=list)


class VerifyActor:
    """One verifier's actor: ``verify_tx`` / ``verify_block`` post messages,
    ``publish`` receives one outcome per message, in mailbox order. ``start``
    runs the loop on a thread; ``stop`` handles every message posted before it
    and joins."""

    def __init__(self, verifier, publish: Callable[[Any], None], config: VerifyActorConfig | None = None):
        self.v = verifier
        self.publish = publish
        self.cfg = config or VerifyActorConfig()
        if self.cfg.max_inputs < 1 or self.cfg.retries < 0:
            raise ValueError("max_inputs >= 1 and retries >= 0")
        self.stats = ActorStats()
        self._q: "queue.Queue" = queue.Queue()
        self._thread: Optional[threading.Thread] = None
        self._crash: Optional[BaseException] = None

    # -- the mailbox ------------------------------------------------------------
    def verify_tx(self, key, tx: bytes, inputs: Sequence[Tuple[int, bytes, int]]) -> None:
        self._post(_Tx(key, tx, list(inputs)))

    def verify_block(self, key, txs: Sequence[bytes], inputs: Sequence[Tuple[int, int, bytes, int]]) -> None:
        self._post(_Block(key, list(txs), list(inputs)))

    def _post(self, msg) -> None:
        if self._crash is not None:
            raise RuntimeError("verify actor stopped on an error") from self._crash
        self._q.put(msg)

    def start(self) -> "VerifyActor":
        if self._thread is None:
            self._thread = threading.Thread(target=self._loop, name="hkv-verify-actor", daemon=True)
            self._thread.start()
        return self

    def stop(self, timeout: float = 600.0) -> None:
        self._q.put(_STOP)
        self.start()
        self._thread.join(timeout)
        if self._thread.is_alive():
            raise TimeoutError("verify actor did not drain its mailbox")
        if self._crash is not None:
            raise self._crash

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    # -- the loop ---------------------------------------------------------------
    def _loop(self) -> None:
        try:
            held = None
            while True:
                msg = held if held is not None else self._q.get()
                held = None
                if msg is _STOP:
                    return
                if isinstance(msg, _Block):
                    self._handle_block(msg)
                    continue
                batch, n = [msg], len(msg.inputs)
                deadline = time.monotonic() + self.cfg.max_wait_s
                while n < self.cfg.max_inputs:
                    try:
                        nxt = self._q.get(timeout=max(0.0, deadline - time.monotonic()))
                    except queue.Empty:
                        break
                    if not isinstance(nxt, _Tx) or n + len(nxt.inputs) > self.cfg.max_inputs:
                        held = nxt
                        break
                    batch.append(nxt)
                    n += len(nxt.inputs)
                self._handle_txs(batch)
        except BaseException as e:  # a bug, not a verify failure: surfaced by stop()
            self._crash = e

    def _verify(self, txs, inputs) -> Tuple[Optional[List[bool]], Optional[str]]:
        err = None
        for _ in range(1 + self.cfg.retries):
            self.stats.gpu_calls += 1
            try:
                ok = verify_std_inputs(self.v, txs, inputs, self.cfg.forkid)
                self.stats.batch_inputs.append(len(inputs))
                return ok, None
            except HkvError as e:
                self.stats.gpu_failures += 1
                err = str(e)
                self.stats.errors.append(err)
        if self.cfg.fallback is not None:
            self.stats.fallback_calls += 1
            try:
                ok = [bool(x) for x in self.cfg.fallback(txs, inputs, self.cfg.forkid)]
            except Exception as e:  # the CPU path failed too: the batch is unverified
                err = f"{err}; fallback: {e!r}"
                self.stats.errors.append(err)
                return None, err
            if len(ok) != len(inputs):
                err = f"{err}; fallback returned {len(ok)} verdicts for {len(inputs)} inputs"
                self.stats.errors.append(err)
                return None, err
            return ok, None
        return None, err

    def _handle_block(self, m: _Block) -> None:
        ok, err = self._verify(m.txs, m.inputs) if m.inputs else ([], None)
        if ok is None:
            self.publish(VerifyFailed(m.key, err))
            return
        bad = tuple((t, i) for (t, i, _, _), v in zip(m.inputs, ok) if not v)
        self.publish(BlockRejected(m.key, bad) if bad else BlockVerified(m.key))

    def _handle_txs(self, batch: List[_Tx]) -> None:
        txs = [m.tx for m in batch]
        inputs = [(k, i, spk, val) for k, m in enumerate(batch) for (i, spk, val) in m.inputs]
        ok, err = self._verify(txs, inputs) if inputs else ([], None)
        at = 0
        for m in batch:
            if ok is None:
                self.publish(VerifyFailed(m.key, err))
                continue
            vs = ok[at: at + len(m.inputs)]
            at += len(m.inputs)
            bad = tuple(i for (i, _, _), v in zip(m.inputs, vs) if not v)
            self.publish(TxRejected(m.key, bad) if bad else TxVerified(m.key))


__all__ = ["VerifyActor", "VerifyActorConfig", "ActorStats", "BlockVerified", "BlockRejected", "TxVerified",
           "TxRejected", "VerifyFailed"]
