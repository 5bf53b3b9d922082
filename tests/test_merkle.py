"""Batch block merkle roots: GPU (hkv_merkle_roots, csrc/hkv_headers.hip)
against the CPU oracle (oracle/merkle_oracle.py), which is pinned by the
reference's own block assertion (test/Haskoin/NodeSpec.hs:185-193:
header merkle == buildMerkleRoot of the txids) on the 15 fixture blocks
(tests/golden/ref_blocks.bin) and by mainnet block 100,000's published root.
"""
import os
import random

import numpy as np
import pytest

import merkle_oracle as mo
from conftest import GOLDEN

# mainnet block 100,000: txids and merkle root in display (reversed) order
B100K_TXIDS = [
    "8c14f0db3df150123e6f3dbbf30f8b955a8249b62ac1d1ff16284aefa3d06d87",
    "fff2525b8931402dd09222c50775608f75787bd2b87e56995a7bdd30f79702c4",
    "6359f0868171b1d194cbee1af2f16ea598ae8fad666d9b012c8ed2b79a236ec4",
    "e9a66845e05d5abc0ad04ec80f774a7e585c6e8db975962d069a522137b80c1d",
]
B100K_ROOT = "f3e94742aca4b5ef85488dc37c06c3282295ffec960994b2c0d5ac2a25a95766"


def internal(display_hex: str) -> bytes:
    return bytes.fromhex(display_hex)[::-1]


def fixture_blocks():
    """(header merkle field, [txid]) of the 15 bchRegTest fixture blocks (one tx each)."""
    raw = open(os.path.join(GOLDEN, "ref_blocks.bin"), "rb").read()
    off, out = 0, []
    while off < len(raw):
        merkle = raw[off + 36:off + 68]
        assert raw[off + 80] == 1
        t0 = off + 81
        off = t0 + 4
        nin = raw[off]; off += 1
        for _ in range(nin):
            off += 36; sl = raw[off]; off += 1 + sl + 4
        nout = raw[off]; off += 1
        for _ in range(nout):
            off += 8; sl = raw[off]; off += 1 + sl
        off += 4
        out.append((merkle, [mo.dsha256(raw[t0:off])]))
    return out


def random_blocks(sizes, seed, dup_frac=0.0):
    rng = random.Random(seed)
    blocks = []
    for n in sizes:
        t = [rng.randbytes(32) for _ in range(n)]
        if n >= 2 and rng.random() < dup_frac:
            i = rng.randrange(0, n - 1) & ~1
            t[i + 1] = t[i]          # a paired duplicate at level 0
        blocks.append(t)
    return blocks


EDGE_SIZES = [0, 1, 2, 3, 4, 5, 7, 8, 255, 256, 257, 511, 512, 513, 1023, 1024, 1025, 2000, 4097]


def test_oracle_reference_fixture_blocks():
    blocks = fixture_blocks()
    assert len(blocks) == 15
    for merkle, txids in blocks:
        root, mut = mo.merkle_root(txids)
        assert root == merkle and not mut


def test_oracle_block_100000():
    root, mut = mo.merkle_root([internal(h) for h in B100K_TXIDS])
    assert root == internal(B100K_ROOT) and not mut


def test_oracle_mutation_flag():
    a, b, c = (bytes([i]) * 32 for i in (1, 2, 3))
    # [a, b, c] and [a, b, c, c] share a root; only the second is mutated
    assert mo.merkle_root([a, b, c])[0] == mo.merkle_root([a, b, c, c])[0]
    assert not mo.merkle_root([a, b, c])[1]
    assert mo.merkle_root([a, b, c, c])[1]
    assert mo.merkle_root([])[0] == bytes(32)


# ---------------------------------------------------------------- GPU -------

@pytest.fixture(scope="module")
def verifier():
    import torch
    import hkv
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    v = hkv.Verifier(hkv.VerifierConfig(device_ids=[0]))
    yield v
    v.close()


@pytest.mark.gpu
def test_gpu_known_answers(verifier):
    import hkv
    fx = fixture_blocks()
    blocks = [t for _, t in fx] + [[internal(h) for h in B100K_TXIDS]]
    roots, mut = hkv.merkle_roots(verifier, blocks)
    assert roots[:15] == [m for m, _ in fx]
    assert roots[15] == internal(B100K_ROOT)
    assert not mut.any()


def _edge_blocks(seed):
    """EDGE_SIZES with level-0 duplicates (dup_frac), an inner-level duplicate
    (6 leaves, level-1 pair equal) and top-join-only duplicates: 16 leaves
    whose second half repeats the first (equal subtree roots; with 8 subtree
    workgroups only hkv_merkle_top_kernel pairs them) and 4,096 leaves with
    the upper 2,048 repeating the lower."""
    rng = random.Random(seed)
    blocks = random_blocks(EDGE_SIZES, seed=seed, dup_frac=0.5)
    t = [rng.randbytes(32) for _ in range(6)]
    t[2], t[3] = t[0], t[1]
    blocks.append(t)
    for n in (16, 4096):
        h = [rng.randbytes(32) for _ in range(n // 2)]
        blocks.append(h + h)
    return blocks


@pytest.mark.gpu
@pytest.mark.parametrize("route", ["split", "full"])
def test_gpu_edge_sizes_parity_both_routes(verifier, route):
    """Batches of at most n_cu (256) blocks take the split route (8 subtree
    workgroups per block + hkv_merkle_top_kernel); larger ones one workgroup
    per block (hkv_merkle_kernel). The same edge blocks go through both: as
    they are (split), and padded with 300 random blocks past the threshold
    (full)."""
    import hkv
    blocks = _edge_blocks(0x4D524B4C)
    pad = random_blocks([1 + k % 9 for k in range(300)], seed=3) if route == "full" else []
    roots, mut = hkv.merkle_roots(verifier, pad + blocks)
    roots, mut = roots[len(pad):], mut[len(pad):]
    for b, t in enumerate(blocks):
        er, em = mo.merkle_root(t)
        assert roots[b] == er, (route, b, len(t))
        assert bool(mut[b]) == em, (route, b, len(t))
    assert mut[-1] and mut[-2] and mut[-3]


@pytest.mark.gpu
def test_gpu_device_form_many_blocks(verifier):
    """4096 HBM-resident blocks of 1..3000 txids (≈6M leaves) through the
    device entry point; a random sample of roots equals the oracle's."""
    import torch
    import hkv
    rng = np.random.default_rng(17)
    nb = 4096
    sizes = rng.integers(1, 3001, size=nb)
    offsets = np.zeros(nb + 1, dtype=np.uint32)
    offsets[1:] = np.cumsum(sizes)
    leaves = rng.integers(0, 256, size=(int(offsets[-1]), 32), dtype=np.uint8)
    dl = torch.from_numpy(leaves.reshape(-1)).cuda()
    do = torch.from_numpy(offsets.view(np.int32).copy()).cuda()
    sc = torch.zeros(int(offsets[-1]) * 32, dtype=torch.uint8, device="cuda")
    dr = torch.zeros(nb * 32, dtype=torch.uint8, device="cuda")
    dm = torch.zeros(nb, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    hkv.merkle_roots_device(verifier, 0, dl.data_ptr(), do.data_ptr(), nb, sc.data_ptr(), dr.data_ptr(),
                            dm.data_ptr(), s)
    torch.cuda.synchronize()
    rb = dr.cpu().numpy().reshape(nb, 32)
    mb = dm.cpu().numpy()
    for b in list(rng.choice(nb, size=40, replace=False)) + [0, nb - 1]:
        t = [leaves[i].tobytes() for i in range(offsets[b], offsets[b + 1])]
        er, em = mo.merkle_root(t)
        assert rb[b].tobytes() == er, b
        assert bool(mb[b]) == em
