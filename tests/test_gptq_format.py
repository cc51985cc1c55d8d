"""AutoGPTQ tensor format: the product's unpackers (quant/gptq.py) against the
oracle's restated AutoGPTQ packer (oracle/gptq_format.py).  auto-gptq itself is not installed and
not vendored: PARITY UNPINNED against the real library — these tests pin the two restatements to
each other and the dequant identity, nothing more."""
import numpy as np
import pytest
import torch

from oracle import gptq_format as OG
from quant import gptq


@pytest.mark.parametrize("bits", [2, 3, 4, 8])
def test_unpack_qweight_roundtrip(bits):
    rs = np.random.RandomState(bits)
    K, N = 32 * 6, 48
    q = rs.randint(0, 2 ** bits, size=(K, N))
    packed = OG.pack_qweight(q, bits)
    assert packed.shape == (K * bits // 32, N)
    got = gptq.unpack_qweight(torch.from_numpy(packed.view(np.int32)), bits)
    assert np.array_equal(got.numpy(), q)


@pytest.mark.parametrize("bits", [2, 3, 4, 8])
def test_unpack_qzeros_roundtrip(bits):
    rs = np.random.RandomState(10 + bits)
    G, N = 5, 32 * 3
    z = rs.randint(1, 2 ** bits, size=(G, N))  # v1 format stores z - 1 in [0, 2^b - 1)
    packed = OG.pack_qzeros(z, bits)
    assert packed.shape == (G, N * bits // 32)
    got = gptq.unpack_qzeros(torch.from_numpy(packed.view(np.int32)), bits, N)
    assert np.array_equal(got.numpy(), z)


@pytest.mark.parametrize("bits,group", [(4, 128), (3, 64), (2, 32), (8, 256)])
def test_dequant_matches_restated_autogptq(bits, group):
    rs = np.random.RandomState(bits * group)
    K, N = 512, 64
    G = K // group
    q = rs.randint(0, 2 ** bits, size=(K, N))
    z = rs.randint(1, 2 ** bits, size=(G, N))
    s = (rs.rand(G, N) * 0.01 + 1e-3).astype(np.float16)
    g_idx = np.arange(K) // group
    ref = OG.dequant(q, z, s, g_idx)
    w = gptq.gptq_dequant(torch.from_numpy(OG.pack_qweight(q, bits).view(np.int32)),
                          torch.from_numpy(OG.pack_qzeros(z, bits).view(np.int32)),
                          torch.from_numpy(s), torch.from_numpy(g_idx.astype(np.int32)), bits)
    assert np.array_equal(w.numpy().view(np.uint16), ref.view(np.uint16))


def test_act_order_rejected():
    K, group = 256, 64
    g = torch.arange(K) // group
    gptq.check_g_idx(g, K, group)
    perm = g[torch.randperm(K, generator=torch.Generator().manual_seed(0))]
    with pytest.raises(NotImplementedError):
        gptq.check_g_idx(perm, K, group)
