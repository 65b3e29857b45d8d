"""CPU: the PLN codec's host logic and transforms.

The device plumbing and the codec itself are checked against the oracle in
test_pln_gpu.py.  Parity of the transforms against TFC is unpinned (no TF, no
checkpoint): these tests pin the properties the restatement declares.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from compression_without_quantization_amd import pln as P


def test_permutations_match_global_seed_sequence(oracle):
    for seed in (0, 42, 2 ** 31 - 1):
        p1, p2 = P.permutations(seed, 1000, 37)
        w1, w2 = oracle.pln_permutations(seed, 1000, 37)
        assert p1.dtype == np.int32 and np.array_equal(p1, w1) and np.array_equal(p2, w2)
    i1, i2 = P.permutations(5, 10, 3, use_permutation=False)
    assert np.array_equal(i1, np.arange(10)) and np.array_equal(i2, np.arange(3))


@pytest.mark.parametrize("hw", [(512, 768), (128, 192), (100, 150)])
def test_transform_shapes(hw):
    m = P.ProbabilisticLadderNetwork(8, 8, 16, 4)
    h, w = hw
    x = torch.rand(1, 3, h, w)
    with torch.no_grad():
        l1, s1 = m.analysis_transform_1(x)
        l2, s2 = m.analysis_transform_2(l1)
        pl, ps = m.synthesis_transform_2(l2)
        r = m.synthesis_transform_1(l1)
    c = lambda n, k: -(-n // k)  # TF 'same': ceil(n / stride)
    assert l1.shape == s1.shape == (1, 16, c(h, 16), c(w, 16))
    assert l2.shape == s2.shape == (1, 4, c(h, 64), c(w, 64))
    assert pl.shape == ps.shape == (1, 16, 4 * c(h, 64), 4 * c(w, 64))
    assert r.shape == (1, 3, 16 * c(h, 16), 16 * c(w, 16))
    assert (s1 > 0).all() and (s2 > 0).all() and (s2 < 1).all() and (ps > 0).all()


def test_kodak_latent_sizes():
    """512x768 -> 32x48x128 (196,608) and 8x12x24 (2,304)."""
    m = P.ProbabilisticLadderNetwork()
    assert m.first_level_latent_channels * 32 * 48 == 196608
    assert m.second_level_latent_channels * 8 * 12 == 2304


def test_gdn_formula():
    torch.manual_seed(0)
    g = P.GDN(5)
    with torch.no_grad():
        g.gamma.copy_(torch.rand(5, 5) * 0.2)
        g.beta.copy_(torch.rand(5) + 0.5)
    x = torch.randn(1, 5, 3, 4)
    y = g(x)
    norm = g.beta.view(1, 5, 1, 1) + torch.einsum("ji,njhw->nihw", g.gamma, x * x)
    assert torch.allclose(y, x / torch.sqrt(norm), rtol=1e-6, atol=1e-7)
    gi = P.GDN(5, inverse=True)
    with torch.no_grad():
        gi.gamma.copy_(g.gamma)
        gi.beta.copy_(g.beta)
    assert torch.allclose(gi(x), x * torch.sqrt(norm), rtol=1e-6, atol=1e-7)


def test_signal_conv_down_is_same_padded_correlation():
    torch.manual_seed(1)
    conv = P.SignalConv2D(2, 3, 5, True, strides_down=2, use_bias=False)
    with torch.no_grad():
        conv.kernel.normal_()
    x = torch.randn(1, 2, 9, 7)
    y = conv(x)
    xp = F.pad(x, (2, 2, 2, 2))
    want = torch.zeros(1, 3, 5, 4)
    for o in range(3):
        for i in range(5):
            for j in range(4):
                patch = xp[0, :, 2 * i:2 * i + 5, 2 * j:2 * j + 5]
                want[0, o, i, j] = (patch * conv.kernel[o]).sum()   # no kernel flip
    assert torch.allclose(y, want, atol=1e-5)


def test_signal_conv_up_is_adjoint_of_down():
    """corr=False with strides_up is the transpose of corr=True with
    strides_down (same kernel): <down(x), y> == <x, up(y)>."""
    torch.manual_seed(2)
    down = P.SignalConv2D(3, 4, 5, True, strides_down=2, use_bias=False)
    up = P.SignalConv2D(4, 3, 5, False, strides_up=2, use_bias=False)
    with torch.no_grad():
        down.kernel.normal_()
        up.kernel.copy_(down.kernel)      # [out=4, in=3] == transposed [in=4, out=3]
    x = torch.randn(1, 3, 16, 12, dtype=torch.float64)
    y = torch.randn(1, 4, 8, 6, dtype=torch.float64)
    down, up = down.double(), up.double()
    lhs = (down(x) * y).sum()
    rhs = (x * up(y)).sum()
    assert torch.allclose(lhs, rhs, rtol=1e-10)


def test_reset_parameters_deterministic():
    a = P.ProbabilisticLadderNetwork(8, 8, 16, 4, init_seed=3)
    b = P.ProbabilisticLadderNetwork(8, 8, 16, 4, init_seed=3)
    c = P.ProbabilisticLadderNetwork(8, 8, 16, 4, init_seed=4)
    sa, sb, sc = a.state_dict(), b.state_dict(), c.state_dict()
    assert all(torch.equal(sa[k], sb[k]) for k in sa)
    assert any(not torch.equal(sa[k], sc[k]) for k in sa)


def test_load_weights_safetensors(tmp_path):
    from safetensors.torch import save_file
    a = P.ProbabilisticLadderNetwork(8, 8, 16, 4, init_seed=3)
    b = P.ProbabilisticLadderNetwork(8, 8, 16, 4, init_seed=9)
    path = str(tmp_path / "w.safetensors")
    save_file({k: v.contiguous() for k, v in a.state_dict().items()}, path)
    b.load_weights(path)
    assert all(torch.equal(a.state_dict()[k], b.state_dict()[k]) for k in a.state_dict())


def test_quantize_image():
    q = P.quantize_image(np.array([-0.1, 0.0, 0.5 / 255, 0.2, 1.0, 1.3], np.float32))
    assert q.dtype == torch.uint8
    assert q.tolist() == [0, 0, 0, 51, 255, 255]   # round half to even, saturate


def test_group_differences_and_counts():
    assert P._group_differences([0, 3, 4, 10]).tolist() == [3, 1, 6]
    with pytest.raises(ValueError):
        P._group_differences([0, 0, 4])                # empty first group -> EOF symbol
    assert P._load_counts("", 17).tolist() == [1] * 17
    assert P._load_counts(None, 5).tolist() == [1] * 5
    assert P._load_counts([3, 0, 2], 5).tolist() == [3, 0, 2]


def test_group_size_coder_roundtrip_uniform_model():
    from compression_without_quantization_amd import ArithmeticCoder
    rng = np.random.default_rng(0)
    diffs = rng.integers(1, 4096, 523)
    ac = ArithmeticCoder(P._load_counts("", 1 + 2 ** 12), 32)
    code = ac.encode(np.concatenate((diffs, [0])))
    assert ac.decode_fast(code)[:-1] == diffs.tolist()


def test_zero_count_symbol_rejected():
    from compression_without_quantization_amd import ArithmeticCoder
    from compression_without_quantization_amd._lib import CwqError
    ac = ArithmeticCoder([1, 0, 5], 32)
    with pytest.raises(CwqError):
        ac.encode([2, 1, 0])


def test_container_extras_layout(tmp_path):
    """pln.py:541-549 extras (11 x 4-byte big-endian) with a negative seed,
    two variable bit strings and four quint16/index lists round trip."""
    from compression_without_quantization_amd import read_bin_code, write_bin_code
    path = str(tmp_path / "x.miracle")
    extras = [-7 & 0xFFFFFFFF, 30, 14, 20, 20, 12, 9, 32, 48, 8, 12]
    vle = [[3, 77], [65535, 1], [], []]
    write_bin_code("101100111010" + "110010011", path, extras=extras,
                   extra_var_bits=[list("1101"), list("0")], var_length_extras=vle,
                   var_length_bits=[24, 16, 24, 16])
    code, ex, evb, v = read_bin_code(path, num_extras=P.NUM_EXTRAS, num_extra_var_bits=2,
                                     num_var_length_extras=4)
    assert ex == extras and evb == ["1101", "0"] and v == vle
    assert code[:21] == "101100111010110010011"
    assert int(np.int32(np.uint32(ex[0]))) == -7
