"""GPU parity tests (MI355X) for the on-device signature hashes and standard
inputs: the HIP kernels through the C
ABI against oracle/sighash_oracle.py — byte-exact hashes, byte-exact verify
records and bit-exact verdicts, including malformed and adversarial inputs."""
import ctypes
import json
import os
import random

import numpy as np
import pytest

import secp256k1_oracle as o
import sighash_oracle as sh
import txgen
from conftest import host_threads, openssl_batch, GOLDEN, oracle_batch

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


def oracle_sighash(raw_txs, jobs, forkid):
    out = []
    for (t, i, code, value, shw, kind) in jobs:
        tx = sh.tx_parse(raw_txs[t])
        if kind == sh.KIND_LEGACY and not (forkid is not None and shw & 0x40) and (shw & 0x1F) == 3 \
                and i >= len(tx.outputs):
            out.append(sh.ONE)
        else:
            out.append(sh.sighash_job(tx, kind, code, value, i, shw, forkid))
    return out


def random_jobs(rng, raw_txs, n_jobs):
    jobs = []
    for _ in range(n_jobs):
        t = rng.randrange(len(raw_txs))
        nin = len(sh.tx_parse(raw_txs[t]).inputs)
        jobs.append((t, rng.randrange(nin), txgen.rand_code(rng), rng.randrange(2**64), txgen.rand_sighash(rng),
                     rng.randrange(2)))
    return jobs


@pytest.mark.parametrize("forkid", [None, 0, 7])
def test_sighash_random_vs_oracle(ver, forkid):
    import hkv
    rng = random.Random(100 + (forkid or 0))
    txs = []
    for k in range(300):
        nin, nout = rng.choice([1, 1, 2, 3, 5, 17]), rng.choice([0, 1, 2, 3, 9])
        txs.append(sh.tx_serialize(txgen.rand_tx(rng, nin, nout, segwit=(k % 3 == 0))))
    txs.append(sh.tx_serialize(txgen.rand_tx(rng, 3, 3, big_scripts=True)))  # 0xFD / 0xFE varints
    jobs = random_jobs(rng, txs, 2500)
    jobs += [(len(txs) - 1, i, txgen.rand_code(rng), 5, s, k) for i in range(3) for s in (1, 2, 3, 0x83)
             for k in (0, 1)]
    got, status = hkv.tx_sig_hash_batch(ver, txs, jobs, forkid)
    exp = oracle_sighash(txs, jobs, forkid)
    assert all(s == 0 for s in status)
    bad = [k for k in range(len(jobs)) if got[k] != exp[k]]
    assert not bad, [(jobs[k][3:], got[k].hex(), exp[k].hex()) for k in bad[:5]]


def test_sighash_bip143_example(ver):
    import hkv
    b = json.load(open(os.path.join(GOLDEN, "bip143_p2wpkh.json")))
    raw = bytes.fromhex(b["unsigned_tx"])
    i0, i1 = b["inputs"]
    h20 = bytes.fromhex(i1["script_pubkey"])[2:]
    got, status = hkv.tx_sig_hash_batch(ver, [raw], [
        (0, 1, sh.p2pkh_script(h20), i1["value"], 1, hkv.HKV_SIGHASH_FORKID),
        (0, 0, bytes.fromhex(i0["script_pubkey"]), i0["value"], 1, hkv.HKV_SIGHASH_LEGACY)])
    assert status == [0, 0]
    assert got[0].hex() == b["input1_sighash_all"]["sigHash"]
    tx = sh.tx_parse(raw)
    assert got[1] == sh.sighash_legacy(tx, bytes.fromhex(i0["script_pubkey"]), 0, 0, 1)


def test_sighash_noncanonical_varints_and_errors(ver):
    import hkv
    rng = random.Random(7)
    tx = txgen.rand_tx(rng, 2, 2)
    tx.outputs[1].script = b"\x76" * 25
    raw = sh.tx_serialize(tx)
    # re-encode output 1's script length 0x19 as FD 19 00 (non-canonical)
    k = raw.rfind(bytes([25]) + b"\x76" * 25)
    nc = raw[:k] + b"\xfd\x19\x00" + raw[k + 1:]
    assert sh.tx_parse(nc).outputs[1].script == b"\x76" * 25
    code = sh.p2pkh_script(b"\x22" * 20)
    jobs = [(0, 0, code, 9, s, kind) for s in (1, 3, 0x81) for kind in (0, 1)]
    got, st = hkv.tx_sig_hash_batch(ver, [nc], jobs)
    assert st == [0] * len(jobs)
    assert got == oracle_sighash([nc], jobs, None)
    assert got == oracle_sighash([raw], jobs, None)  # haskoin hashes the re-serialised tx
    # errors: truncated tx, input out of range, tx index out of range
    trunc = raw[:-5]
    got, st = hkv.tx_sig_hash_batch(ver, [trunc, raw], [(0, 0, code, 0, 1, 0), (1, 2, code, 0, 1, 0),
                                                        (1, 1, code, 0, 1, 1)])
    assert st == [hkv.lib.HKV_SH_BAD_TX, hkv.lib.HKV_SH_BAD_INPUT, 0]
    assert got[0] == b"\0" * 32 and got[1] == b"\0" * 32
    # the ABI rejects a job that points past the batch only per job (status), not the call
    from hkv.sighash import SIGHASH_JOB_DTYPE, TxBatch
    tb = TxBatch([raw])
    arr = np.zeros(2, dtype=SIGHASH_JOB_DTYPE)
    arr[0] = (5, 0, 0, 0, 0, 1, 0)
    arr[1] = (0, 0, 0, 10_000, 0, 1, 0)
    st_, pool = tb.struct()
    out = np.zeros((2, 32), dtype=np.uint8)
    status = np.zeros(2, dtype=np.uint8)
    assert ver.lib.hkv_sighash(ver.ctx, ctypes.byref(st_), arr.ctypes.data, 2, -1, out.ctypes.data,
                               status.ctypes.data) == 0
    assert list(status) == [3, 3]


# --- standard inputs -----------------------------------------------------------

def upload(torch, arr: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8).copy()).cuda()


def device_std_records(torch, ver, raw_txs, inputs, forkid):
    """Run hkv_std_inputs_device and return the 168-byte records."""
    import hkv
    from hkv.sighash import INPUT_JOB_DTYPE, TxBatch
    tb = TxBatch(raw_txs)
    arr = np.zeros(len(inputs), dtype=INPUT_JOB_DTYPE)
    for k, (t, i, spk, value) in enumerate(inputs):
        off, ln = tb.script(spk)
        arr[k] = (t, i, off, ln, value)
    _, pool = tb.struct()
    d_bytes, d_off, d_pool, d_jobs = upload(torch, tb.bytes), upload(torch, tb.offsets), upload(torch, pool), \
        upload(torch, arr)
    dt = hkv.HkvTxs(d_bytes.data_ptr(), d_off.data_ptr(), len(raw_txs), d_pool.data_ptr(), tb._len)
    recs = torch.zeros(len(inputs) * 168, dtype=torch.uint8, device="cuda")
    ver.std_inputs_device(0, dt, d_jobs.data_ptr(), len(inputs), -1 if forkid is None else forkid, recs.data_ptr())
    torch.cuda.synchronize()
    return recs.cpu().numpy().tobytes()


def mutate_block(rng, txs, jobs, forkid):
    """Adversarial copies of signed inputs (one mutation each)."""
    out_txs, out_jobs, kinds = [], [], []
    p2sh_jobs = [j for j in jobs if len(j[2]) == 23]
    for m in range(17):
        pool = p2sh_jobs if m >= 14 else jobs
        for (t, i, prev, val) in rng.sample(pool, min(6, len(pool))):
            tx = sh.tx_parse(sh.tx_serialize(txs[t]))
            seg = len(prev) in (22, 23)
            sig = tx.witness[i][0] if seg else sh._push_items(tx.inputs[i].script)[0]
            pub = tx.witness[i][1] if seg else (sh._push_items(tx.inputs[i].script) + [b""])[1]
            r, s = sh.sig_parse_der(sig[:-1])
            if m == 0:
                sig = sig[:5] + bytes([sig[5] ^ 1]) + sig[6:]           # r byte flipped: ECDSA fails
            elif m == 1:
                sig = sh.der_encode(r, o.N - s) + sig[-1:]              # high S: strict decode fails
            elif m == 2:
                sig = sig[:-1] + b"\x04"                                 # unknown hashtype
            elif m == 3:
                sig = sig[:-1] + b"\x41"                                 # FORKID byte
            elif m == 4:
                sig = sig[:1] + b"\x81" + sig[1:2] + sig[2:]            # long-form length < 128
            elif m == 5:
                sig = sig + b"\x00"                                      # trailing byte (after hashtype)
            elif m == 6:
                pub = txgen.Key(rng.randrange(1, o.N)).pub               # HASH160 mismatch
            elif m == 7:
                prev = prev[:-1] + b"\x00"                               # not a template
            elif m == 8:
                val += 1                                                 # wrong amount (BIP143 only)
            elif m == 9:
                sig = sh.der_encode(r, s) + b"\x03"                      # SIGHASH_SINGLE: other msg
            elif m == 10:
                sig = sig[:-1] + b"\x81"                                 # ANYONECANPAY|ALL: other msg
            elif m == 11:
                sig = b"\x30\x06\x02\x01\x00\x02\x01\x01\x01"           # r = 0
            elif m == 12:
                sig = sh.der_encode(o.N + 5, s) + sig[-1:]               # r >= n -> 0 -> reject
            if seg:
                tx.witness[i] = [sig, pub] if m != 13 else [sig, pub, b""]   # 13: 3 witness items
                if m == 14:                                                   # P2SH: two pushes
                    tx.inputs[i].script = tx.inputs[i].script * 2
                elif m == 15:                                                 # P2SH: other program
                    tx.inputs[i].script = txgen.push(sh.p2wpkh_script(rng.randbytes(20)))
                elif m == 16:                                                 # P2SH: empty scriptSig
                    tx.inputs[i].script = b""
            else:
                tx.inputs[i].script = txgen.push(sig) + (txgen.push(pub) if pub else b"") + \
                    (b"\x51" if m == 13 else b"")                        # 13: trailing OP_1
            out_txs.append(sh.tx_serialize(tx))
            out_jobs.append((len(out_txs) - 1, i, prev, val))
            kinds.append(m)
    return out_txs, out_jobs, kinds


@pytest.mark.parametrize("forkid", [None, 0])
def test_std_inputs_records_and_verdicts_vs_oracle(torch, ver, coracle, forkid):
    import hkv
    rng = random.Random(31 + (forkid or 0))
    keys = [txgen.Key(rng.randrange(1, o.N), compressed=(k % 5 != 0)) for k in range(16)]
    txs, jobs = txgen.std_block(rng, 60, keys, forkid=forkid, p2wpkh_share=0.4, p2pk_share=0.2, p2sh_share=0.2)
    raw = [sh.tx_serialize(t) for t in txs]
    mtx, mjobs, kinds = mutate_block(rng, txs, jobs, forkid)
    all_raw = raw + mtx
    all_jobs = jobs + [(t + len(raw), i, p, v) for (t, i, p, v) in mjobs]
    recs = device_std_records(torch, ver, all_raw, all_jobs, forkid)
    exp = b"".join(sh.std_input_record(sh.tx_parse(all_raw[t]), i, p, v, forkid) for (t, i, p, v) in all_jobs)
    bad = [k for k in range(len(all_jobs)) if recs[k * 168:(k + 1) * 168] != exp[k * 168:(k + 1) * 168]]
    assert not bad, [(k, kinds[k - len(jobs)] if k >= len(jobs) else "valid") for k in bad[:10]]
    verdicts = hkv.verify_std_inputs(ver, all_raw, all_jobs, forkid)
    want = oracle_batch(coracle, exp, 1)
    assert verdicts == want.tolist()
    assert all(verdicts[:len(jobs)])             # every generated input verifies
    rej = [not v for v in verdicts[len(jobs):]]
    assert sum(rej) > 0.8 * len(rej)             # nearly every mutation is rejected (oracle decides which)


@pytest.mark.parametrize("forkid", [None, 0])
def test_std_inputs_block_kernel_small_batches(torch, ver, coracle, forkid):
    """Batches of 1, 2, 15, 16, 17, 31, 33 and 100 standard inputs take the
    block kernel (hkv_block_kernel<true>: 16 inputs per workgroup, three chain
    segments, LDS-flag hand-offs, a 16-bit verdict store per workgroup):
    partial last workgroups and bitmap half-words shared by two workgroups.
    Verdicts through the host and the device entry points equal the oracle's
    on the records the oracle derives; a flipped signature byte rejects
    exactly its input."""
    import hkv
    rng = random.Random(77 + (forkid or 0))
    keys = [txgen.Key(rng.randrange(1, o.N), compressed=(k % 4 != 0)) for k in range(8)]
    txs, jobs = txgen.std_block(rng, 90, keys, forkid=forkid, p2wpkh_share=0.4, p2pk_share=0.2, p2sh_share=0.2)
    raw = [sh.tx_serialize(t) for t in txs]
    parsed = [sh.tx_parse(t) for t in raw]
    assert len(jobs) >= 100
    for n in (1, 2, 15, 16, 17, 31, 33, 100):
        sub = jobs[:n]
        exp = b"".join(sh.std_input_record(parsed[t], i, p, v, forkid) for (t, i, p, v) in sub)
        want = oracle_batch(coracle, exp, 1).tolist()
        assert all(want)
        assert hkv.verify_std_inputs(ver, raw, sub, forkid) == want
        assert _device_verify_std(torch, ver, raw, sub, forkid) == want
    # one bad input in the middle of a 33-input batch (workgroup 1, bit 16 of word 0 / half-word 1)
    t, i, p, v = jobs[20]
    tx = sh.tx_parse(raw[t])
    bad = list(raw)
    if tx.witness and tx.witness[i]:
        w = list(tx.witness[i])
        w[0] = w[0][:7] + bytes([w[0][7] ^ 0x10]) + w[0][8:]
        tx.witness[i] = w
    else:
        items = sh._push_items(tx.inputs[i].script)
        items[0] = items[0][:7] + bytes([items[0][7] ^ 0x10]) + items[0][8:]
        tx.inputs[i].script = b"".join(txgen.push(x) for x in items)
    bad[t] = sh.tx_serialize(tx)
    got = hkv.verify_std_inputs(ver, bad, jobs[:33], forkid)
    expect = [True] * 33
    for k, (tk, ik, _, _) in enumerate(jobs[:33]):
        if tk == t and ik == i:
            expect[k] = False
    assert got == expect


@pytest.mark.parametrize("forkid", [None, 0])
def test_block_kernel_large_txs_vs_oracle(torch, ver, coracle, forkid):
    """The block kernel copies each input's tx to LDS when it fits in 2 KB
    (hkv_kernels.hip TxCache, TXC_WORDS) and builds the tx index rows itself;
    larger txs are parsed, indexed and hashed from HBM. A block of 24-, 14-
    and 2-input txs (the 24-input ones past 2 KB, the 14-input ones around
    it) verifies like the oracle through both entry points, and a flipped
    signature byte in a large tx rejects exactly that input."""
    import hkv
    rng = random.Random(5150 + (forkid or 0))
    keys = [txgen.Key(rng.randrange(1, o.N), compressed=(k % 4 != 0)) for k in range(8)]
    txs, jobs = txgen.std_block(rng, 6, keys, forkid=forkid, p2wpkh_share=0.3, p2pk_share=0.2, p2sh_share=0.2,
                                nin_choices=(24, 14, 2))
    raw = [sh.tx_serialize(t) for t in txs]
    assert max(len(r) for r in raw) > 2048
    parsed = [sh.tx_parse(t) for t in raw]
    exp = b"".join(sh.std_input_record(parsed[t], i, p, v, forkid) for (t, i, p, v) in jobs)
    want = oracle_batch(coracle, exp, 1).tolist()
    assert all(want) and len(jobs) <= 4096
    assert hkv.verify_std_inputs(ver, raw, jobs, forkid) == want
    assert _device_verify_std(torch, ver, raw, jobs, forkid) == want
    # flip one signature byte of an input of the largest tx
    big = max(range(len(raw)), key=lambda k: len(raw[k]))
    t, i, p, v = next(j for j in jobs if j[0] == big and j[1] == 7)
    tx = sh.tx_parse(raw[t])
    if tx.witness and tx.witness[i]:
        w = list(tx.witness[i])
        w[0] = w[0][:7] + bytes([w[0][7] ^ 0x10]) + w[0][8:]
        tx.witness[i] = w
    else:
        items = sh._push_items(tx.inputs[i].script)
        items[0] = items[0][:7] + bytes([items[0][7] ^ 0x10]) + items[0][8:]
        tx.inputs[i].script = b"".join(txgen.push(x) for x in items)
    bad = list(raw)
    bad[t] = sh.tx_serialize(tx)
    got = _device_verify_std(torch, ver, bad, jobs, forkid)
    assert got == [not (jt == t and ji == i) for (jt, ji, _, _) in jobs]


def test_std_inputs_bip143_example(ver):
    import hkv
    b = json.load(open(os.path.join(GOLDEN, "bip143_p2wpkh.json")))
    tx = sh.tx_parse(bytes.fromhex(b["unsigned_tx"]))
    i0, i1 = b["inputs"]
    tx.inputs[0].script = txgen.push(bytes.fromhex(i0["sig"]))
    tx.witness = [[], [bytes.fromhex(i1["sig"]), bytes.fromhex(i1["pubkey"])]]
    raw = sh.tx_serialize(tx)
    jobs = [(0, k, bytes.fromhex(x["script_pubkey"]), x["value"]) for k, x in enumerate(b["inputs"])]
    assert hkv.verify_std_inputs(ver, [raw], jobs) == [True, True]
    jobs_bad = [(0, k, s, v + 1) for (_, k, s, v) in jobs]
    assert hkv.verify_std_inputs(ver, [raw], jobs_bad) == [True, False]  # only BIP143 commits to the amount


def test_gen_keys_and_sign(torch, ver, coracle):
    n = 300
    priv = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    pub = torch.zeros(n * 33, dtype=torch.uint8, device="cuda")
    h160 = torch.zeros(n * 20, dtype=torch.uint8, device="cuda")
    ver.gen_keys_device(0, 99, n, priv.data_ptr(), pub.data_ptr(), h160.data_ptr())
    msgs = torch.randint(0, 256, (n * 32,), dtype=torch.uint8, device="cuda")
    idx = torch.arange(n, dtype=torch.int32, device="cuda").flip(0).contiguous()
    sig = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
    ver.gen_sign_device(0, 5, n, priv.data_ptr(), idx.data_ptr(), msgs.data_ptr(), 32, sig.data_ptr())
    torch.cuda.synchronize()
    P, Q, H, M, S = (x.cpu().numpy().tobytes() for x in (priv, pub, h160, msgs, sig))
    recs = []
    for k in range(n):
        d = int.from_bytes(P[32 * k:32 * k + 32], "big")
        pk = Q[33 * k:33 * k + 33]
        assert o.pubkey_serialize(o.point_mul(d, o.G), True) == pk
        assert sh.hash160(pk) == H[20 * k:20 * k + 20]
        j = n - 1 - k  # signature j uses key idx[j] = n-1-j
        recs.append(o.make_record(M[32 * j:32 * j + 32], S[64 * j:64 * j + 64], pk))
    assert oracle_batch(coracle, b"".join(recs), 0).all()


def _block_vs_oracle(torch, ver, coracle, openssl, txs, inputs):
    """Every input's 168-byte verify record (msg32 = the sighash, r, s, key)
    equals the oracle's std_input_record (Python txSigHash / decodeTxSig /
    HASH160 restatement); verdicts equal the C restatement and OpenSSL."""
    import hkv
    got = hkv.verify_std_inputs(ver, txs, inputs)
    recs = device_std_records(torch, ver, txs, inputs, None)
    parsed = [sh.tx_parse(t) for t in txs]
    exp = b"".join(sh.std_input_record(parsed[t], i, p, v) for (t, i, p, v) in inputs)
    bad = [k for k in range(len(inputs)) if recs[k * 168:(k + 1) * 168] != exp[k * 168:(k + 1) * 168]]
    assert not bad, bad[:10]
    assert got == oracle_batch(coracle, exp, 1, threads=host_threads()).tolist()
    assert got == openssl_batch(openssl, exp, 1, threads=host_threads()).tolist()
    return got


def test_block_mix_config3_all_valid(torch, ver, coracle, openssl):
    """BASELINE configs[2]: 2,000-tx P2PKH + P2WPKH block from the product-side
    generator verifies end to end; EVERY input's record is re-derived by the
    oracle (so a sighash bug shared by signer and verifier cannot hide)."""
    from hkv import blockgen
    txs, inputs = blockgen.make_block(ver, torch, n_tx=2000)
    assert 3000 < len(inputs) < 5000
    assert all(_block_vs_oracle(torch, ver, coracle, openssl, txs, inputs))


def test_p2pkh_block_config0(torch, ver, coracle, openssl):
    """BASELINE configs[0]: 2,000 txs x 2 P2PKH inputs x 2 P2PKH outputs =
    4,000 signatures (seed 0x484B5631, 4,096-key pool, compressed keys,
    SIGHASH_ALL): every record byte-exact against the oracle, every verdict
    accepted and equal to both CPU checkers; one mutated input per tx
    (a flipped scriptSig signature byte) rejects exactly those inputs."""
    from hkv import blockgen
    txs, inputs = blockgen.make_p2pkh_block(ver, torch)
    assert len(txs) == 2000 and len(inputs) == 4000
    assert all(len(p) == 25 for (_, _, p, _) in inputs)
    assert all(_block_vs_oracle(torch, ver, coracle, openssl, txs, inputs))
    rng = random.Random(0x484B5631)
    bad_txs, flips = [], []
    for t, raw in enumerate(txs):
        tx = sh.tx_parse(raw)
        i = rng.randrange(2)
        items = sh._push_items(tx.inputs[i].script)
        sig = items[0]
        sig = sig[:7] + bytes([sig[7] ^ 0x10]) + sig[8:]  # a byte of r: ECDSA (or DER) must reject
        tx.inputs[i].script = txgen.push(sig) + txgen.push(items[1])
        bad_txs.append(sh.tx_serialize(tx))
        flips.append(2 * t + i)
    got = _block_vs_oracle(torch, ver, coracle, openssl, bad_txs, inputs)
    assert [k for k, v in enumerate(got) if not v] == flips


# --- multisig (bare and P2SH) ---------------------------------------------------

def _ms_oracle(coracle, txs, jobs, forkid):
    from test_sighash_oracle import multisig_verdicts
    return multisig_verdicts(coracle, [sh.tx_parse(t) for t in txs], jobs, forkid)


def _device_verify_std(torch, ver, raw_txs, inputs, forkid, records=False, status=False):
    """hkv_verify_std_inputs_device over HBM-resident txs / jobs (records:
    also the 168-byte records the call wrote; status: through
    hkv_verify_std_inputs_device_status, also the call's status word)."""
    import hkv
    from hkv.sighash import INPUT_JOB_DTYPE, TxBatch
    tb = TxBatch(raw_txs)
    arr = np.zeros(len(inputs), dtype=INPUT_JOB_DTYPE)
    for k, (t, i, spk, value) in enumerate(inputs):
        off, ln = tb.script(spk)
        arr[k] = (t, i, off, ln, value)
    _, pool = tb.struct()
    d_bytes, d_off, d_pool, d_jobs = upload(torch, tb.bytes), upload(torch, tb.offsets), upload(torch, pool), \
        upload(torch, arr)
    dt = hkv.HkvTxs(d_bytes.data_ptr(), d_off.data_ptr(), len(raw_txs), d_pool.data_ptr(), tb._len)
    recs = torch.zeros(len(inputs) * 168, dtype=torch.uint8, device="cuda")
    bits = torch.zeros(((len(inputs) + 63) // 64) * 2, dtype=torch.int32, device="cuda")
    st = torch.zeros(2, dtype=torch.int32, device="cuda")
    ver.verify_std_inputs_device(0, dt, d_jobs.data_ptr(), len(inputs), -1 if forkid is None else forkid,
                                 recs.data_ptr(), bits.data_ptr(), d_status=st.data_ptr() if status else 0)
    torch.cuda.synchronize()
    w = bits.cpu().numpy().view(np.uint32)
    got = [bool((w[k // 32] >> (k % 32)) & 1) for k in range(len(inputs))]
    if status:
        return got, int(st[0].item())
    return (got, recs.cpu().numpy().tobytes()) if records else got


@pytest.mark.parametrize("n_fill,forkid", [(20000, None), (20000, 0), (2600, None), (75000, None)])
def test_std_inputs_full_grid_overlap_vs_oracle(torch, ver, coracle, n_fill, forkid):
    """Above 32,768 inputs the extraction overlaps the ECDSA kernels
    (hkv_api.cpp enqueue_std_chunk): the parse half writes the records the
    prologue and the Q chains read, the hash half rewrites them whole on a
    second stream, and u1 is formed after the join (hkv_late_u1_kernel).
    Every mutation class of mutate_block — including those only the hash half
    decides (HASH160 mismatch, a wrong BIP143 amount, the SINGLE and
    ANYONECANPAY messages) — spread through a ~37,000-input batch: the final
    records of the generated and mutated inputs are byte-exact against the
    oracle's, every verdict equals the C oracle's on the records the call
    wrote, and the host entry point agrees. With a 2,600-tx filler (~4,900
    inputs) the same batch takes the fused pair kernel instead; with a
    75,000-tx filler (~138,000 inputs) it runs as two chunks (131,072 inputs
    through the overlapped form, the rest through the pair kernel) on one
    stream, sharing the index rows and the fork / join events."""
    import hkv
    from hkv import blockgen
    rng = random.Random(4242 + (forkid or 0))
    keys = [txgen.Key(rng.randrange(1, o.N), compressed=(k % 5 != 0)) for k in range(16)]
    txs, jobs = txgen.std_block(rng, 60, keys, forkid=forkid, p2wpkh_share=0.4, p2pk_share=0.2, p2sh_share=0.2)
    raw = [sh.tx_serialize(t) for t in txs]
    mtx, mjobs, _ = mutate_block(rng, txs, jobs, forkid)
    small_raw = raw + mtx
    small_jobs = jobs + [(t + len(raw), i, p, v) for (t, i, p, v) in mjobs]
    exp_small = [sh.std_input_record(sh.tx_parse(small_raw[t]), i, p, v, forkid) for (t, i, p, v) in small_jobs]
    btxs, bjobs = blockgen.make_block(ver, torch, n_tx=n_fill, seed=blockgen.SEED + 99 + n_fill)
    all_raw = btxs + small_raw
    all_jobs = list(bjobs) + [(t + len(btxs), i, p, v) for (t, i, p, v) in small_jobs]
    order = list(range(len(all_jobs)))
    rng.shuffle(order)
    jobs_sh = [all_jobs[k] for k in order]
    assert len(jobs_sh) > (131072 if n_fill >= 75000 else 32768 if n_fill >= 20000 else 16 * 256)
    got, recs = _device_verify_std(torch, ver, all_raw, jobs_sh, forkid, records=True)
    bad = [pos for pos, k in enumerate(order)
           if k >= len(bjobs) and recs[pos * 168:(pos + 1) * 168] != exp_small[k - len(bjobs)]]
    assert not bad, bad[:10]
    want = oracle_batch(coracle, recs, 1).tolist()
    assert got == want
    small_got = [None] * len(small_jobs)
    for pos, k in enumerate(order):
        if k >= len(bjobs):
            small_got[k - len(bjobs)] = got[pos]
    assert sum(small_got[:len(jobs)]) == len(jobs)                  # every generated input verifies
    assert len(small_got) - sum(small_got) > 0.8 * len(mjobs)        # nearly every mutation rejects
    if forkid is None:
        assert all(got[pos] for pos, k in enumerate(order) if k < len(bjobs))
    assert hkv.verify_std_inputs(ver, all_raw, jobs_sh, forkid) == got


@pytest.mark.parametrize("forkid", [None, 0])
def test_multisig_inputs_vs_oracle(torch, ver, coracle, forkid):
    """Bare, P2SH, P2WSH and P2SH-P2WSH m-of-n inputs (1-of-1 .. 15-of-15,
    1-of-16; up to 22 valid and adversarial variants, tests/txgen.py
    multisig_cases) shuffled into a
    signed single-signature block: verdicts of the host and device entry
    points equal the oracle's countMulSig walk over C-oracle candidate
    verdicts, and the single-signature inputs are unaffected."""
    import hkv
    rng = random.Random(177 + (forkid or 0))
    keys = [txgen.Key(rng.randrange(1, o.N), compressed=(k % 4 != 0)) for k in range(24)]
    mtxs, mjobs, names = txgen.multisig_cases(rng, keys, forkid)
    btxs, bjobs = txgen.std_block(rng, 40, keys, forkid=forkid, p2wpkh_share=0.4, p2pk_share=0.2, p2sh_share=0.2)
    raw = [sh.tx_serialize(t) for t in btxs + mtxs]
    jobs = bjobs + [(t + len(btxs), i, p, v) for (t, i, p, v) in mjobs]
    labels = ["single"] * len(bjobs) + names
    order = list(range(len(jobs)))
    rng.shuffle(order)
    jobs = [jobs[k] for k in order]
    labels = [labels[k] for k in order]
    want = _ms_oracle(coracle, raw, jobs, forkid)
    got = hkv.verify_std_inputs(ver, raw, jobs, forkid)
    bad = [(labels[k], got[k], want[k]) for k in range(len(jobs)) if got[k] != want[k]]
    assert not bad, bad[:10]
    assert _device_verify_std(torch, ver, raw, jobs, forkid) == got
    assert all(g for g, lb in zip(got, labels) if lb == "single")
    assert sum(got) > len(bjobs) + 80
    assert {lb.split("-")[0] for lb in labels} == {"single", "bare", "p2sh", "p2wsh", "p2sh_p2wsh"}


def test_multisig_many_inputs(torch, ver, coracle):
    """600 P2SH 2-of-3 inputs (every third with one signature corrupted) in
    one batch: record ranges allocated per input on device, verdicts equal
    the oracle's."""
    import hkv
    rng = random.Random(4242)
    keys = [txgen.Key(rng.randrange(1, o.N)) for _ in range(12)]
    txs, jobs = [], []
    for t in range(600):
        ks = rng.sample(keys, 3)
        script = txgen.multisig_script(2, [k.pub for k in ks])
        tx = sh.Tx(2, [sh.TxIn(txgen.rand_script(rng, 32), 0, b"", 0xFFFFFFFF)],
                   [sh.TxOut(1000 + t, sh.p2pkh_script(txgen.rand_script(rng, 20)))], [[]], 0)
        msg = sh.sighash_legacy(tx, script, 5000, 0, 1)
        idx = sorted(rng.sample(range(3), 2))
        items = []
        for k in idx:
            r, s = txgen.sign(msg, ks[k].d if (t % 3 or k != idx[1]) else ks[k].d + 1, rng.randrange(1, o.N))
            items.append(sh.der_encode(r, s) + b"\x01")
        tx.inputs[0].script = b"\x00" + b"".join(txgen.push(x) for x in items) + txgen.push(script)
        txs.append(sh.tx_serialize(tx))
        jobs.append((t, 0, txgen.p2sh_script(script), 5000))
    got = hkv.verify_std_inputs(ver, txs, jobs)
    assert got == _ms_oracle(coracle, txs, jobs, None)
    assert got == [t % 3 != 0 for t in range(600)]


@pytest.mark.parametrize("forkid", [None, 0])
def test_wrapped_single_sig_vs_oracle(torch, ver, coracle, forkid):
    """P2SH-P2PK / P2SH-P2PKH / P2WSH-P2PK / P2WSH-P2PKH / P2SH-P2WSH-P2PK /
    P2SH-P2WSH-P2PKH inputs, valid and mutated (tests/txgen.py
    wrapped_single_cases): every 168-byte record byte-exact against the
    oracle's std_input_record (sighash over the redeem / witness script, the
    script-hash checks), verdicts equal to the oracle on the host and device
    entry points."""
    import hkv
    rng = random.Random(299 + (forkid or 0))
    keys = [txgen.Key(rng.randrange(1, o.N), compressed=(k % 3 != 0)) for k in range(8)]
    txs, jobs, names = txgen.wrapped_single_cases(rng, keys, forkid)
    raw = [sh.tx_serialize(t) for t in txs]
    recs = device_std_records(torch, ver, raw, jobs, forkid)
    exp = b"".join(sh.std_input_record(txs[t], i, p, v, forkid) for (t, i, p, v) in jobs)
    bad = [names[k] for k in range(len(jobs)) if recs[k * 168:(k + 1) * 168] != exp[k * 168:(k + 1) * 168]]
    assert not bad, bad[:10]
    want = _ms_oracle(coracle, raw, jobs, forkid)
    got = hkv.verify_std_inputs(ver, raw, jobs, forkid)
    assert got == want, [(names[k], got[k], want[k]) for k in range(len(jobs)) if got[k] != want[k]][:10]
    assert _device_verify_std(torch, ver, raw, jobs, forkid) == got
    assert sum(got) >= 6 * 4 and len(got) - sum(got) >= 6 * 5


def _ms_mix(rng, forkid):
    keys = [txgen.Key(rng.randrange(1, o.N), compressed=(k % 4 != 0)) for k in range(24)]
    mtxs, mjobs, names = txgen.multisig_cases(rng, keys, forkid)
    return [sh.tx_serialize(t) for t in mtxs], mjobs, names


@pytest.mark.parametrize("n_tx,forkid", [(3000, None), (3000, 0), (20000, None)])
def test_multisig_on_every_launch_shape(torch, ver, coracle, n_tx, forkid):
    """The multisig cases (bare, P2SH, P2WSH, P2SH-P2WSH; valid and
    adversarial) inside batches past the block kernel's bound: ~5,500 inputs
    take the fused pair kernel with the separate scan kernel (that
    path had no multisig GPU test), ~37,000 the extraction kernel and the
    full-grid verify. Host and device entry points: the multisig verdicts
    equal the oracle's countMulSig walk, every generated single-signature
    input verifies."""
    import hkv
    from hkv import blockgen
    rng = random.Random(1313 + n_tx + (forkid or 0))
    btxs, bjobs = blockgen.make_block(ver, torch, n_tx=n_tx, seed=blockgen.SEED + 7 * n_tx)
    mraw, mjobs, names = _ms_mix(rng, forkid)
    raw = btxs + mraw
    jobs = list(bjobs) + [(t + len(btxs), i, p, v) for (t, i, p, v) in mjobs]
    order = list(range(len(jobs)))
    rng.shuffle(order)
    jobs = [jobs[k] for k in order]
    is_ms = [k >= len(bjobs) for k in order]
    assert len(jobs) > 16 * 256
    want_ms = _ms_oracle(coracle, mraw, mjobs, forkid)
    want = [None] * len(jobs)
    for pos, k in enumerate(order):
        want[pos] = want_ms[k - len(bjobs)] if k >= len(bjobs) else True
    got = hkv.verify_std_inputs(ver, raw, jobs, forkid)
    if forkid is None:
        bad = [(names[order[p] - len(bjobs)] if is_ms[p] else "single", got[p], want[p])
               for p in range(len(jobs)) if got[p] != want[p]]
        assert not bad, bad[:10]
    else:  # the device generator's singles sign without the fork id: only the multisig verdicts are meaningful
        bad = [(names[order[p] - len(bjobs)], got[p], want[p]) for p in range(len(jobs)) if is_ms[p] and got[p] != want[p]]
        assert not bad, bad[:10]
    assert _device_verify_std(torch, ver, raw, jobs, forkid) == got
    assert sum(g for g, m in zip(got, is_ms) if m) > 80


def test_std_inputs_device_returns_before_the_stream_runs(torch, ver, coracle):
    """hkv_verify_std_inputs_device only enqueues: with
    the call's stream gated behind ~20 full-grid verifies on another stream
    (an event wait), the call returns long before the gate opens, and once it
    has run the verdicts — multisig inputs included, whose count the host
    never reads — equal the oracle's."""
    import time
    import hkv
    from hkv.sighash import INPUT_JOB_DTYPE, TxBatch
    rng = random.Random(2024)
    mraw, mjobs, _ = _ms_mix(rng, None)
    keys = [txgen.Key(rng.randrange(1, o.N)) for _ in range(8)]
    btxs, bjobs = txgen.std_block(rng, 40, keys, p2wpkh_share=0.4, p2pk_share=0.2, p2sh_share=0.2)
    raw = [sh.tx_serialize(t) for t in btxs] + mraw
    jobs = list(bjobs) + [(t + len(btxs), i, p, v) for (t, i, p, v) in mjobs]
    want = _ms_oracle(coracle, raw, jobs, None)
    tb = TxBatch(raw)
    arr = np.zeros(len(jobs), dtype=INPUT_JOB_DTYPE)
    for k, (t, i, spk, value) in enumerate(jobs):
        off, ln = tb.script(spk)
        arr[k] = (t, i, off, ln, value)
    _, pool = tb.struct()
    d_bytes, d_off, d_pool, d_jobs = upload(torch, tb.bytes), upload(torch, tb.offsets), upload(torch, pool), \
        upload(torch, arr)
    dt = hkv.HkvTxs(d_bytes.data_ptr(), d_off.data_ptr(), len(raw), d_pool.data_ptr(), tb._len)
    recs = torch.zeros(len(jobs) * 168, dtype=torch.uint8, device="cuda")
    bits = torch.zeros(((len(jobs) + 63) // 64) * 2, dtype=torch.int32, device="cuda")
    # the gate: full-grid verifies of 1M records on another stream, ~9 ms each
    n_big = 1 << 20
    big = torch.empty(n_big * 168, dtype=torch.uint8, device="cuda")
    bbits = torch.zeros(n_big // 32 + 2, dtype=torch.int32, device="cuda")
    ver.gen_records_device(0, 77, n_big, 4096, 100, big.data_ptr())
    gate, s = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        ver.verify_device(0, big.data_ptr(), n_big, 0, bbits.data_ptr(), gate.cuda_stream)
    ev = torch.cuda.Event()
    ev.record(gate)
    s.wait_event(ev)
    t1 = time.perf_counter()
    ver.verify_std_inputs_device(0, dt, d_jobs.data_ptr(), len(jobs), -1, recs.data_ptr(), bits.data_ptr(),
                                 s.cuda_stream)
    t_call = time.perf_counter() - t1
    torch.cuda.synchronize()
    t_gate = time.perf_counter() - t0
    assert t_gate > 0.1, t_gate
    assert t_call < 0.25 * t_gate, (t_call, t_gate)
    w = bits.cpu().numpy().view(np.uint32)
    got = [bool((w[k // 32] >> (k % 32)) & 1) for k in range(len(jobs))]
    assert got == want
    assert int(bbits[: n_big // 32].cpu().numpy().view(np.uint32).astype(np.uint64).sum()) == (n_big // 32) * 0xFFFFFFFF


def _ms_block(rng, forkid, n_single=40):
    """A block-kernel-sized batch: tx 0 a coinbase no input spends (no job
    references it, so the block kernel builds no index row for it), signed
    single-signature txs and the multisig cases, shuffled."""
    keys = [txgen.Key(rng.randrange(1, o.N), compressed=(k % 4 != 0)) for k in range(24)]
    mtxs, mjobs, names = txgen.multisig_cases(rng, keys, forkid)
    btxs, bjobs = txgen.std_block(rng, n_single, keys, forkid=forkid, p2wpkh_share=0.4, p2pk_share=0.2,
                                  p2sh_share=0.2)
    cb = sh.Tx(1, [sh.TxIn(b"\0" * 32, 0xFFFFFFFF, b"\x03\x01\x02\x03", 0xFFFFFFFF)],
               [sh.TxOut(50 * 10**8, sh.p2wpkh_script(b"\x11" * 20))], [[b"\0" * 32]], 0)
    raw = [sh.tx_serialize(cb)] + [sh.tx_serialize(t) for t in btxs + mtxs]
    jobs = [(t + 1, i, p, v) for (t, i, p, v) in bjobs] + [(t + 1 + len(btxs), i, p, v) for (t, i, p, v) in mjobs]
    labels = ["single"] * len(bjobs) + names
    order = list(range(len(jobs)))
    rng.shuffle(order)
    return raw, [jobs[k] for k in order], [labels[k] for k in order]


@pytest.mark.parametrize("forkid", [None, 0])
def test_tail_hashes_txs_no_input_references(torch, ver, coracle, forkid):
    """the multisig tail hashes every tx of the batch
    (BIP143 per-tx hashes), but the block kernel builds index rows only for
    the txs its inputs reference — a block's coinbase has none. The rows
    are left over from an earlier call over a much larger tx buffer (a
    sighash batch of large witness txs, so the stale rows carry TXF_OK |
    TXF_WITNESS and offsets far past this batch's buffer). The tail now
    re-derives each row from the offsets: verdicts equal the oracle's
    through both entry points, and again after a second stale fill."""
    import hkv
    rng = random.Random(9090 + (forkid or 0))
    raw, jobs, labels = _ms_block(rng, forkid)
    assert len(jobs) <= 16 * 256 and all(t != 0 for (t, _, _, _) in jobs)
    want = _ms_oracle(coracle, raw, jobs, forkid)
    big = [sh.tx_serialize(txgen.rand_tx(rng, 40, 30, segwit=True)) for _ in range(len(raw) + 8)]
    for rep in range(2):
        sj = [(t, 0, b"\x51", 1, 1, 1) for t in range(len(big))]
        hkv.tx_sig_hash_batch(ver, big, sj, forkid)  # fills the txt rows of every tx index of this batch
        got = _device_verify_std(torch, ver, raw, jobs, forkid)
        bad = [(labels[k], got[k], want[k]) for k in range(len(jobs)) if got[k] != want[k]]
        assert not bad, bad[:10]
        hkv.tx_sig_hash_batch(ver, big, sj, forkid)
        assert hkv.verify_std_inputs(ver, raw, jobs, forkid) == want
    assert sum(g for g, lb in zip(want, labels) if lb != "single") > 40


def test_tail_barrier_fault_reported_then_clean(torch, ver, coracle):
    """VERDICT r04 item 3 / ADVICE r04: a multisig tail whose grid barrier
    gives up (forced by the HKV_FAIL_TAIL hook) reports the fault through
    the device form's status word, the device's sticky latch
    (hkv_device_fault, read-and-clear) and the host form's return code
    (HKV_E_INTERNAL); its multisig verdicts are rejects only (never an
    accept the oracle does not give), the single-signature verdicts are
    untouched, and the next call — whose barrier uses the other slot,
    which the faulted launch zeroed — is bit-exact again with no fault."""
    import hkv
    from hkv.lib import HKV_FAIL_TAIL, HKV_STATUS_TAIL_FAULT, HkvError
    rng = random.Random(5151)
    raw, jobs, labels = _ms_block(rng, None)
    want = _ms_oracle(coracle, raw, jobs, None)
    assert ver.device_fault(0) == 0
    # the device form with a status word
    assert ver.lib.hkv_debug_fail_device(ver.ctx, 0, HKV_FAIL_TAIL) == 0
    got, st = _device_verify_std(torch, ver, raw, jobs, None, status=True)
    assert st == HKV_STATUS_TAIL_FAULT
    assert all(w or not g for g, w in zip(got, want))            # no false accept
    assert all(g == w for g, w, lb in zip(got, want, labels) if lb == "single")
    assert any(w and not g for g, w in zip(got, want))           # the fault cost some multisig accepts
    assert ver.device_fault(0) == HKV_STATUS_TAIL_FAULT
    assert ver.device_fault(0) == 0                              # read-and-clear
    got, st = _device_verify_std(torch, ver, raw, jobs, None, status=True)
    assert st == 0 and got == want
    # the plain device form: the latch only
    assert ver.lib.hkv_debug_fail_device(ver.ctx, 0, HKV_FAIL_TAIL) == 0
    got = _device_verify_std(torch, ver, raw, jobs, None)
    assert all(w or not g for g, w in zip(got, want))
    assert ver.device_fault(0) == HKV_STATUS_TAIL_FAULT
    # the host form: its own call's status
    assert ver.lib.hkv_debug_fail_device(ver.ctx, 0, HKV_FAIL_TAIL) == 0
    with pytest.raises(HkvError) as ei:
        hkv.verify_std_inputs(ver, raw, jobs)
    assert ei.value.rc == -5
    assert hkv.verify_std_inputs(ver, raw, jobs) == want         # an earlier fault is not this call's
    assert _device_verify_std(torch, ver, raw, jobs, None) == want
    assert ver.device_fault(0) == HKV_STATUS_TAIL_FAULT          # (the host-form fault above)
    assert ver.device_fault(0) == 0


# --- malformed wire data on the block kernel's LDS tx view ----------------------

def _segments(tx):
    """The wire form of tx as named segments (so a test can rewrite one
    field — a count, a length varint — and keep the rest byte-exact)."""
    seg = any(len(w) for w in tx.witness)
    out = [("ver", tx.version.to_bytes(4, "little"))]
    if seg:
        out.append(("marker", b"\x00\x01"))
    out.append(("nin", sh.put_varint(len(tx.inputs))))
    for j, ti in enumerate(tx.inputs):
        out += [(f"in{j}_op", ti.outpoint()), (f"in{j}_sl", sh.put_varint(len(ti.script))), (f"in{j}_s", ti.script),
                (f"in{j}_seq", ti.sequence.to_bytes(4, "little"))]
    out.append(("nout", sh.put_varint(len(tx.outputs))))
    for k, to in enumerate(tx.outputs):
        out += [(f"out{k}_v", to.value.to_bytes(8, "little")), (f"out{k}_sl", sh.put_varint(len(to.script))),
                (f"out{k}_s", to.script)]
    if seg:
        for j, w in enumerate(tx.witness):
            out.append((f"w{j}_n", sh.put_varint(len(w))))
            for q, item in enumerate(w):
                out += [(f"w{j}_{q}_l", sh.put_varint(len(item))), (f"w{j}_{q}", item)]
    out.append(("lock", tx.locktime.to_bytes(4, "little")))
    assert b"".join(b for _, b in out) == sh.tx_serialize(tx)
    return out


def _rewrite(tx, name, new):
    return b"".join(new if n == name else b for n, b in _segments(tx))


def _padded(rng, keys, kind, target, forkid=None):
    """A signed one-job tx of exactly `target` bytes: input 0 spends a
    `kind` prevout, input 1 is padding whose scriptSig neither sighash form
    commits to (legacy blanks the other inputs' scripts, BIP143 hashes only
    their outpoints and sequences), grown after signing to hit the size."""
    while True:
        txs, jobs = txgen.std_block(rng, 1, keys, forkid=forkid, nin_choices=(2,),
                                    p2wpkh_share=1.0 if kind == "p2wpkh" else 0.0)
        tx = txs[0]
        if kind == "p2pkh" and len(jobs[0][2]) != 25:
            continue
        tx.inputs[1].script = b""
        base = len(sh.tx_serialize(tx))
        for pad in range(max(0, target - base - 4), target - base + 1):
            if base + pad + len(sh.put_varint(pad)) - 1 == target:
                tx.inputs[1].script = b"\x6a" * pad
                raw = sh.tx_serialize(tx)
                assert len(raw) == target
                return tx, raw, jobs[0]


@pytest.mark.parametrize("forkid", [None, 0])
def test_block_kernel_malformed_wire_vs_oracle(torch, ver, coracle, forkid):
    """VERDICT r04 item 4 (after the round-4 aperture violation on the block
    kernel's LDS tx view): at block size, through both standard-input entry
    points, txs whose wire form lies — truncated at several points, input /
    output counts and scriptSig / output-script / witness varints (1-, 3-,
    5- and 9-byte forms) that claim more bytes than the tx holds, a tx of
    under 10 bytes and an empty one — beside valid txs of exactly 2,047,
    2,048 (the LDS copy's limit) and 2,049 bytes, a 2,049-byte tx cut to
    2,048, a prevout script that ends at the script pool's last byte and a
    job whose script range runs past the pool. Every verdict equals the
    oracle's (a tx that does not parse rejects), and every record the block
    kernel wrote equals the oracle's (all-zero for a reject)."""
    import hkv
    from hkv.sighash import INPUT_JOB_DTYPE, TxBatch
    rng = random.Random(2049 + (forkid or 0))
    keys = [txgen.Key(rng.randrange(1, o.N), compressed=(k % 4 != 0)) for k in range(8)]
    txs, jobs = txgen.std_block(rng, 30, keys, forkid=forkid, p2wpkh_share=0.4, p2pk_share=0.2, p2sh_share=0.2)
    raw = [sh.tx_serialize(t) for t in txs]
    jobs = list(jobs)
    names = ["valid"] * len(jobs)

    def add(b, job, name):
        raw.append(b)
        jobs.append((len(raw) - 1,) + tuple(job[1:]))
        names.append(name)

    # the signed txs the mutations start from: every template of std_block
    bases = [(txs[t], (t, i, p, v)) for (t, i, p, v) in jobs[:12]]
    big = [b"\xfd\xff\xff", b"\xfe\xff\xff\xff\xff", b"\xff" + b"\xff" * 8, b"\xfe\x00\x00\x01\x00"]
    for bt, job in bases:
        b = sh.tx_serialize(bt)
        for cut in (1, 4, 5, len(b) // 2, len(b) - 9):
            add(b[:-cut], job, f"trunc{cut}")
        i = job[1]
        segs = dict(_segments(bt))
        add(_rewrite(bt, "nin", sh.put_varint(len(bt.inputs) + 1)), job, "nin+1")
        add(_rewrite(bt, "nout", sh.put_varint(len(bt.outputs) + 1)), job, "nout+1")
        add(_rewrite(bt, f"in{i}_sl", sh.put_varint(len(bt.inputs[i].script) + 1)), job, "sl+1")
        add(_rewrite(bt, "out1_sl", sh.put_varint(len(bt.outputs[1].script) + 5)), job, "osl+5")
        for v in big:
            add(_rewrite(bt, "nin", v), job, "nin_big")
            add(_rewrite(bt, "nout", v), job, "nout_big")
            add(_rewrite(bt, f"in{i}_sl", v), job, "sl_big")
            add(_rewrite(bt, "out0_sl", v), job, "osl_big")
        if f"w{i}_n" in segs:
            for v in big[:2]:
                add(_rewrite(bt, f"w{i}_n", v), job, "wn_big")
                add(_rewrite(bt, f"w{i}_0_l", v), job, "wl_big")
            add(_rewrite(bt, f"w{i}_n", sh.put_varint(len(bt.witness[i]) + 1)), job, "wn+1")
    add(b"\x01\x00\x00\x00\x01\x00", bases[0][1], "short")
    add(b"", bases[0][1], "empty")
    for kind in ("p2pkh", "p2wpkh"):
        for size in (2047, 2048, 2049):
            _, b, job = _padded(rng, keys, kind, size, forkid)
            add(b, (None,) + tuple(job[1:]), f"{kind}_{size}")
        _, b, job = _padded(rng, keys, kind, 2049, forkid)
        add(b[:2048], (None,) + tuple(job[1:]), f"{kind}_2049_cut")
    # the last job's prevout script is new, so it ends the pool
    kz = txgen.Key(rng.randrange(1, o.N))
    ztx, zjobs = txgen.std_block(rng, 1, [kz], forkid=forkid, nin_choices=(1,), p2wpkh_share=0.0)
    add(sh.tx_serialize(ztx[0]), (None,) + tuple(zjobs[0][1:]), "pool_end")
    assert len(jobs) <= 16 * 256

    parsed = []
    for b in raw:
        try:
            parsed.append(sh.tx_parse(b))
        except (ValueError, IndexError):
            parsed.append(None)
    exp = [sh.std_input_record(parsed[t], i, p, v, forkid) if parsed[t] is not None else b"\0" * 168
           for (t, i, p, v) in jobs]
    want = oracle_batch(coracle, b"".join(exp), 1).tolist()
    for n, w in zip(names, want):
        if n == "valid" or n[-4:] in ("2047", "2048", "2049") or n == "pool_end":
            assert w, n
    assert sum(not w for w in want) > 100

    def check(got, recs=None):
        bad = [(names[k], got[k], want[k]) for k in range(len(jobs)) if got[k] != want[k]]
        assert not bad, bad[:10]
        if recs is not None:
            badr = [names[k] for k in range(len(jobs)) if recs[k * 168:(k + 1) * 168] != exp[k]]
            assert not badr, badr[:10]

    check(hkv.verify_std_inputs(ver, raw, jobs, forkid))
    check(*_device_verify_std(torch, ver, raw, jobs, forkid, records=True))
    # the pool-end job: its script is the pool's last bytes; a job whose range
    # runs past the pool (or wraps) rejects
    tb = TxBatch(raw)
    arr = np.zeros(len(jobs) + 2, dtype=INPUT_JOB_DTYPE)
    for k, (t, i, spk, value) in enumerate(jobs):
        off, ln = tb.script(spk)
        arr[k] = (t, i, off, ln, value)
    assert arr[len(jobs) - 1]["script_off"] + arr[len(jobs) - 1]["script_len"] == tb._len
    last = arr[len(jobs) - 1]
    arr[len(jobs)] = (last["tx"], last["input"], last["script_off"] + 1, last["script_len"], last["value"])
    arr[len(jobs) + 1] = (last["tx"], last["input"], 0xFFFFFFF0, 0x20, last["value"])
    st, pool = tb.struct()
    words = np.zeros((len(arr) + 31) // 32, dtype=np.uint32)
    rc = ver.lib.hkv_verify_std_inputs(ver.ctx, ctypes.byref(st), arr.ctypes.data, len(arr),
                                       -1 if forkid is None else forkid,
                                       words.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    assert rc == 0
    from hkv.records import unpack_bits
    got = unpack_bits(words, len(arr)).tolist()
    check(got[:len(jobs)])
    assert got[len(jobs):] == [False, False]


def test_block_kernel_random_wire_mutations_vs_oracle(torch, ver, coracle):
    """Random byte-level damage to signed txs (a byte flipped, inserted or
    deleted at a random position, the tail cut, two txs spliced), 1,500
    mutants in one block-sized batch beside their intact originals, through
    both standard-input entry points: every verdict equals the oracle's
    (a tx that no longer parses rejects) and every record the block kernel
    wrote equals the oracle's. Complements the structured malformed-wire
    cases with positions the structure does not pick."""
    _wire_mutation_batch(torch, ver, coracle, 0xF022)


def _wire_mutation_batch(torch, ver, coracle, seed, n_mut=1500):
    """One block-sized batch of n_mut random wire mutants (seeded) beside
    their originals: GPU verdicts and records == the oracle's, both forms."""
    import hkv
    rng = random.Random(seed)
    keys = [txgen.Key(rng.randrange(1, o.N), compressed=(k % 4 != 0)) for k in range(8)]
    txs, jobs = txgen.std_block(rng, 120, keys, p2wpkh_share=0.4, p2pk_share=0.2, p2sh_share=0.2)
    raw = [sh.tx_serialize(t) for t in txs]
    all_raw, all_jobs, kinds = list(raw), list(jobs), ["valid"] * len(jobs)
    for _ in range(n_mut):
        t, i, p, v = rng.choice(jobs)
        b = bytearray(raw[t])
        k = rng.randrange(6)
        pos = rng.randrange(len(b))
        if k == 0:
            b[pos] ^= 1 << rng.randrange(8)
        elif k == 1:
            b.insert(pos, rng.randrange(256))
        elif k == 2:
            del b[pos]
        elif k == 3:
            b = b[:pos]
        elif k == 4:
            b[pos] = rng.choice([0x00, 0xFD, 0xFE, 0xFF])
        else:
            other = raw[rng.randrange(len(raw))]
            b = b[:pos] + other[rng.randrange(len(other)):]
        all_raw.append(bytes(b))
        all_jobs.append((len(all_raw) - 1, i, p, v))
        kinds.append(("flip", "insert", "delete", "cut", "varint", "splice")[k])
    assert len(all_jobs) <= 16 * 256
    parsed = []
    for b in all_raw:
        try:
            parsed.append(sh.tx_parse(b))
        except (ValueError, IndexError):
            parsed.append(None)
    exp = []
    for (t, i, p, v) in all_jobs:
        tx = parsed[t]
        ok = tx is not None and i < len(tx.inputs)
        exp.append(sh.std_input_record(tx, i, p, v, None) if ok else b"\0" * 168)
    want = oracle_batch(coracle, b"".join(exp), 1).tolist()
    assert all(want[:len(jobs)]) and sum(not w for w in want) > 1000
    got, recs = _device_verify_std(torch, ver, all_raw, all_jobs, None, records=True)
    bad = [(kinds[k], got[k], want[k]) for k in range(len(all_jobs)) if got[k] != want[k]]
    assert not bad, bad[:10]
    badr = [kinds[k] for k in range(len(all_jobs)) if recs[k * 168:(k + 1) * 168] != exp[k]]
    assert not badr, badr[:10]
    assert hkv.verify_std_inputs(ver, all_raw, all_jobs) == want


@pytest.mark.skipif(not os.environ.get("HKV_STRESS_SEEDS"), reason="stress run only (HKV_STRESS_SEEDS=n)")
def test_block_kernel_wire_mutation_stress(torch, ver, coracle):
    """The mutation batch above over HKV_STRESS_SEEDS further seeds, from
    seed index HKV_STRESS_SEED0 (default 0; a stress run outside the suite:
    profiles/r05o/, r06h/, r06q/)."""
    k0 = int(os.environ.get("HKV_STRESS_SEED0", "0"))
    for k in range(int(os.environ["HKV_STRESS_SEEDS"])):
        _wire_mutation_batch(torch, ver, coracle, 0x5EED0000 + k0 + k)
        if k % 20 == 19:
            print(f"wire mutation stress: {k + 1} batches ({(k + 1) * 1500} mutants, seeds from {k0}) match",
                  flush=True)


@pytest.mark.skipif(not os.environ.get("HKV_STRESS_MS_BLOCKS"), reason="stress run only (HKV_STRESS_MS_BLOCKS=n)")
def test_multisig_block_stress(torch, ver, coracle):
    """Opt-in stress (profiles/r05q/): n seeded block-kernel batches, each a
    coinbase no input spends, signed single-signature inputs and every
    multisig case of txgen (bare / P2SH / P2WSH / P2SH-P2WSH, m-of-n, wrong
    order, bad keys, NULLDUMMY), fork id alternating: device-form verdicts
    (and every fifth batch the host form) equal the oracle's on every input,
    and no call reports a tail fault. HKV_STRESS_MS_WINDOW=c,k runs every
    batch with the tail's record windows forced to c candidate / k key-check
    records (hkv_debug_ms_window: many rounds per batch); HKV_STRESS_SEED0
    starts at a later batch seed."""
    import hkv
    k0 = int(os.environ.get("HKV_STRESS_SEED0", "0"))
    win = os.environ.get("HKV_STRESS_MS_WINDOW")
    if win:
        c, kk = (int(x) for x in win.split(","))
        assert ver.lib.hkv_debug_ms_window(ver.ctx, 0, c, kk) == 0
    for k in range(k0, k0 + int(os.environ["HKV_STRESS_MS_BLOCKS"])):
        forkid = None if k % 2 == 0 else 0
        raw, jobs, labels = _ms_block(random.Random(0x4D530000 + k), forkid)
        want = _ms_oracle(coracle, raw, jobs, forkid)
        got, st = _device_verify_std(torch, ver, raw, jobs, forkid, status=True)
        bad = [(labels[j], got[j], want[j]) for j in range(len(jobs)) if got[j] != want[j]]
        assert not bad and st == 0, (k, st, bad[:10])
        if k % 5 == 0:
            assert hkv.verify_std_inputs(ver, raw, jobs, forkid) == want, k
        print(f"multisig block stress: {k + 1} batches ({len(jobs)} inputs) match", flush=True)
    if win:
        assert ver.lib.hkv_debug_ms_window(ver.ctx, 0, 0, 0) == 0
    assert ver.device_fault(0) == 0
