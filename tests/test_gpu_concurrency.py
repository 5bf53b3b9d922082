"""Concurrent callers on one context (SURVEY §8(b) Threading: one hkv_ctx
per process, calls serialised per device, concurrent calls queued; a
-threaded Haskell node calls through `foreign import ccall safe` from any OS
thread). Python threads release the GIL inside every ctypes call, so the
calls below really overlap in libhkv: host-form and device-form entry
points, record batches and standard-input blocks with multisig inputs (whose
scan sums and tail queue slots alternate per call), each device-form caller
on its own stream. Every call must return its own batch's verdicts."""
import os
import random
import threading

import numpy as np
import pytest

from test_gpu_sighash import _ms_block, _ms_oracle, upload

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need the MI355X"
    return t


@pytest.fixture(scope="module")
def ver(torch):
    import hkv
    v = hkv.Verifier(hkv.VerifierConfig(device_ids=[0], flags=1))
    yield v
    v.close()


def _device_block(torch, raw_txs, inputs):
    """The block's txs / jobs in HBM (read-only, shared by the callers)."""
    import hkv
    from hkv.sighash import INPUT_JOB_DTYPE, TxBatch
    tb = TxBatch(raw_txs)
    arr = np.zeros(len(inputs), dtype=INPUT_JOB_DTYPE)
    for k, (t, i, spk, value) in enumerate(inputs):
        off, ln = tb.script(spk)
        arr[k] = (t, i, off, ln, value)
    _, pool = tb.struct()
    keep = [upload(torch, tb.bytes), upload(torch, tb.offsets), upload(torch, pool), upload(torch, arr)]
    dt = hkv.HkvTxs(keep[0].data_ptr(), keep[1].data_ptr(), len(raw_txs), keep[2].data_ptr(), tb._len)
    return dt, keep


def _bits(torch, w, n):
    words = w.cpu().numpy().view(np.uint32)
    return np.unpackbits(words.view(np.uint8), bitorder="little")[:n].astype(bool)


def test_threads_share_one_context(torch, ver, coracle):
    import hkv
    rounds = int(os.environ.get("HKV_STRESS_ROUNDS", "4"))  # (a longer stress run: HKV_STRESS_ROUNDS=40)
    # record batches: generated valid records, every third one's r corrupted
    n = 70_000
    d_a = torch.empty(n * 168, dtype=torch.uint8, device="cuda")
    ver.gen_records_device(0, 0x434F4E43, n, 65536, 100, d_a.data_ptr())
    torch.cuda.synchronize()
    host_a = d_a.cpu().numpy().copy()
    host_b = host_a.copy()
    host_b.reshape(-1, 168)[::3, 40] ^= 0x01
    want_a = np.ones(n, dtype=bool)
    want_b = want_a.copy()
    want_b[::3] = False
    d_b = torch.from_numpy(host_b).cuda()
    # two standard-input blocks with multisig inputs (block-kernel sized), and
    # their oracle verdicts
    blocks = []
    for seed, forkid in ((0x5101, None), (0x5102, 0)):
        raw, jobs, _ = _ms_block(random.Random(seed), forkid)
        blocks.append((raw, jobs, forkid, _ms_oracle(coracle, raw, jobs, forkid)))
    dev_blocks = [_device_block(torch, raw, jobs) for raw, jobs, _, _ in blocks]

    errors, done = [], []

    def run(name, fn):
        try:
            for r in range(rounds):
                fn(r)
            done.append(name)
        except Exception as e:  # noqa: BLE001 (reported below)
            errors.append((name, repr(e)))

    def host_records(host, want, mode):
        def f(_):
            got = ver.verify_records(host, mode)
            assert (got == want).all(), int((got != want).sum())
        return f

    def device_records(d, want):
        s = torch.cuda.Stream()
        bits = torch.zeros((n + 63) // 64 * 2, dtype=torch.int32, device="cuda")

        def f(_):
            bits.zero_()
            torch.cuda.synchronize()
            ver.verify_device(0, d.data_ptr(), n, 0, bits.data_ptr(), s.cuda_stream)
            s.synchronize()
            got = _bits(torch, bits, n)
            assert (got == want).all(), int((got != want).sum())
        return f

    def device_block(k):
        raw, jobs, forkid, want = blocks[k]
        dt, _ = dev_blocks[k]
        s = torch.cuda.Stream()
        m = len(jobs)
        recs = torch.zeros(m * 168, dtype=torch.uint8, device="cuda")
        bits = torch.zeros((m + 63) // 64 * 2, dtype=torch.int32, device="cuda")
        status = torch.zeros(2, dtype=torch.int32, device="cuda")

        def f(_):
            bits.zero_()
            status.zero_()
            torch.cuda.synchronize()
            ver.verify_std_inputs_device(0, dt, dev_blocks[k][1][3].data_ptr(), m, -1 if forkid is None else forkid,
                                         recs.data_ptr(), bits.data_ptr(), s.cuda_stream, d_status=status.data_ptr())
            s.synchronize()
            got = _bits(torch, bits, m)
            assert int(status[0].item()) == 0
            bad = [j for j in range(m) if got[j] != want[j]]
            assert not bad, bad[:10]
        return f

    def host_block(k):
        raw, jobs, forkid, want = blocks[k]

        def f(_):
            got = hkv.verify_std_inputs(ver, raw, jobs, forkid)
            bad = [j for j in range(len(jobs)) if got[j] != want[j]]
            assert not bad, bad[:10]
        return f

    callers = [("host_records_a", host_records(host_a, want_a, 0)),
               ("host_records_b", host_records(host_b, want_b, 1)),
               ("device_records_b", device_records(d_b, want_b)),
               ("device_block_0", device_block(0)),
               ("device_block_1", device_block(1)),
               ("host_block_1", host_block(1))]
    threads = [threading.Thread(target=run, args=c, daemon=True) for c in callers]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=max(90, 20 * rounds))
    assert not any(t.is_alive() for t in threads), "a caller did not return (deadlock?)"
    assert not errors, errors
    assert sorted(done) == sorted(name for name, _ in callers)
    assert ver.device_fault(0) == 0
