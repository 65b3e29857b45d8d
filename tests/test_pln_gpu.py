"""GPU: the PLN codec against the oracle.

* the HIP latent plumbing (csrc/cwq_pln.hip) bit-exactly against numpy float32;
* code_image_greedy's coded samples against the oracle's grouped coders run
  on the same latent distributions (the transforms' outputs are taken from the
  model itself: TFC parity is unpinned, the coding around them is not);
* decode_image_greedy(file) reproduces the encoder's samples and
  reconstruction bit for bit.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def P(cwqlib):
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = True
    from compression_without_quantization_amd import pln
    return pln


def _bits(a):
    return np.ascontiguousarray(np.asarray(a, np.float32)).view(np.uint32)


def _eq(got, want, what):
    g, w = _bits(got).reshape(-1), _bits(want).reshape(-1)
    bad = np.nonzero(g != w)[0]
    assert g.size == w.size and bad.size == 0, f"{what}: {bad.size} of {w.size} differ"


def test_posterior_combine_vs_numpy(P, oracle):
    rng = np.random.default_rng(3)
    n = 100_003
    ll = rng.standard_normal(n).astype(np.float32)
    ls = np.exp(rng.uniform(-8, 3, n)).astype(np.float32)
    pl = rng.standard_normal(n).astype(np.float32) * 3
    ps = np.exp(rng.uniform(-8, 3, n)).astype(np.float32)
    ls[:4] = [1e-30, 1e-7, 1e19, 0.0]      # eps-dominated, huge and zero scales
    ps[4:8] = [1e-30, 1e-7, 1e19, 0.0]
    d = lambda a: torch.from_numpy(a).cuda()
    loc, scale = P.posterior_combine(d(ll), d(ls), d(pl), d(ps))
    wl, ws = oracle.pln_posterior(ll, ls, pl, ps)
    _eq(loc.cpu().numpy(), wl, "posterior loc")
    _eq(scale.cpu().numpy(), ws, "posterior scale")


@pytest.mark.parametrize("shape", [(1, 128, 32, 48), (1, 24, 8, 12), (1, 5, 3, 7)])
def test_permute_flatten_and_inverse(P, oracle, shape):
    rng = np.random.default_rng(4)
    x = rng.standard_normal(shape).astype(np.float32)
    n = x.size
    perm, _ = oracle.pln_permutations(42, n, 1)
    pd = torch.from_numpy(perm).cuda()
    got = P.permute_flatten(torch.from_numpy(x).cuda(), pd).cpu().numpy()
    _eq(got, oracle.nhwc_permute_flatten(x, perm), "gather")
    back = P.unpermute_unflatten(torch.from_numpy(got).cuda(), pd, shape).cpu().numpy()
    _eq(back, x, "scatter(gather(x))")
    ident = P.permute_flatten(torch.from_numpy(x).cuda(), None).cpu().numpy()
    _eq(ident, np.transpose(x, (0, 2, 3, 1)).reshape(-1), "NHWC flatten")


def _image(h, w, seed=0):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w] / max(h, w)
    base = np.stack([np.sin(6 * xx + c) * np.cos(4 * yy - c) for c in range(3)], -1)
    img = 0.5 + 0.35 * base + 0.05 * rng.standard_normal((h, w, 3))
    return np.clip(img, 0, 1).astype(np.float32)[None]


def _model(P, seed=0, **kw):
    args = dict(first_level_filters=32, second_level_filters=16, first_level_latent_channels=32,
                second_level_latent_channels=8, init_seed=seed)
    args.update(kw)
    return P.ProbabilisticLadderNetwork(**args).cuda().eval()


def _imp_decoder_view(oracle, ind, st, oi, oq, pl, ps, seed):
    """What decode_grouped_importance_sample reconstructs (:337-361): coded
    rows destandardised, dequantised outliers where non-zero."""
    n = pl.size
    z, o = np.zeros(n, np.float32), np.ones(n, np.float32)
    coded = np.zeros(n, np.float32)
    for g, (a, b) in enumerate(zip(st[:-1], st[1:])):
        coded[a:b] = oracle.importance_decode_block(ind[g] - 1, z[a:b], o[a:b], seed + g)
    coded = oracle.destandardise(coded, pl, ps)
    upd = np.zeros(n, np.float32)
    upd[np.asarray(oi, np.int64)] = oracle.dequantize_quint16(oq)
    return np.where(upd == 0, coded, upd).astype(np.float32)


def _oracle_levels(P, oracle, model, img, seed, kw, level1):
    """The codec restated on the oracle: latents from the model, coding on the
    CPU.  Returns the encoder's samples and the decoder's level-1 view."""
    lat = model.latent_distributions(img, seed)
    q1, q2 = lat["q1"], lat["q2"]
    s1, s2 = tuple(q1.loc.shape), tuple(q2.loc.shape)
    perm1, perm2 = oracle.pln_permutations(seed, int(np.prod(s1)), int(np.prod(s2)))
    f = lambda t, p: oracle.nhwc_permute_flatten(t.cpu().numpy(), p)
    q2l, q2s = f(q2.loc, perm2), f(q2.scale, perm2)
    n2 = q2l.size
    z, o = np.zeros(n2, np.float32), np.ones(n2, np.float32)
    samp2, ind2, st2, (oi2, oq2) = oracle.code_grouped_importance_sample(
        q2l, q2s, z, o, seed, kw["second_level_n_bits_per_group"],
        kw["second_level_max_group_size_bits"], kw["second_level_dim_kl_bit_limit"])
    dec2 = _imp_decoder_view(oracle, ind2, st2, oi2, oq2, z, o, seed)
    z2 = torch.from_numpy(oracle.unpermute_to_nchw(dec2, perm2, s2)).cuda()
    with torch.no_grad():
        pl1, ps1 = model.synthesis_transform_2(z2)
    p1l, p1s = f(pl1, perm1), f(ps1, perm1)
    q1l, q1s = f(q1.loc, perm1), f(q1.scale, perm1)
    if level1 == "greedy":
        from compression_without_quantization_amd import group_size_threshold
        samp1, idx1, st1 = oracle.code_grouped_greedy_sample(
            q1l, q1s, p1l, p1s, kw["n_steps"], kw["n_bits_per_step"], seed,
            group_size_threshold(kw["greedy_max_group_size_bits"]))
        dec1 = samp1
    else:
        samp1, ind1, st1, (oi1, oq1) = oracle.code_grouped_importance_sample(
            q1l, q1s, p1l, p1s, seed, kw["first_level_n_bits_per_group"],
            kw["first_level_max_group_size_bits"], kw["first_level_dim_kl_bit_limit"])
        dec1 = _imp_decoder_view(oracle, ind1, st1, oi1, oq1, p1l, p1s, seed)
    return samp2, st2, samp1, st1, dec1, perm1, s1


KW = dict(n_steps=2, n_bits_per_step=8, greedy_max_group_size_bits=12,
          second_level_n_bits_per_group=12, second_level_max_group_size_bits=2,
          second_level_dim_kl_bit_limit=10, first_level_n_bits_per_group=12,
          first_level_max_group_size_bits=4, first_level_dim_kl_bit_limit=10)


@pytest.mark.parametrize("level1", ["greedy", "importance"])
def test_codec_vs_oracle_and_roundtrip(P, oracle, tmp_path, level1):
    model = _model(P, seed=1)
    img = _image(128, 192, seed=1)
    seed = 42
    path = str(tmp_path / "img.miracle")
    (sample2, sample1), summ = model.code_image_greedy(
        None, img, seed, comp_file_path=path,
        use_importance_sampling=(level1 == "importance"), **KW)
    w2, wst2, w1, wst1, dec1, perm1, s1 = _oracle_levels(P, oracle, model, img, seed, KW,
                                                          level1)
    _eq(sample2, w2, "level-2 sample")
    _eq(sample1, w1, "level-1 sample")
    assert summ["actual_byte_size"] > 0 and summ["second_level_groups"] == len(wst2)
    rec = model.decode_image_greedy(None, path, use_importance_sampling=(level1 == "importance"),
                                    greedy_max_group_size_bits=12,
                                    first_level_max_group_size_bits=4,
                                    second_level_max_group_size_bits=2)
    assert rec.shape == (128, 192, 3)
    # the decoder reconstructs SynthesisTransform_1 of the level-1 sample it
    # decodes, which the oracle predicts from the file's contents
    z1 = P.unpermute_unflatten(torch.from_numpy(dec1).cuda(), torch.from_numpy(perm1).cuda(), s1)
    with torch.no_grad():
        want = model.synthesis_transform_1(z1)[0].permute(1, 2, 0).cpu().numpy()
    _eq(rec, want, "reconstruction")


def test_codec_file_is_deterministic(P, tmp_path):
    model = _model(P, seed=2)
    img = _image(64, 128, seed=2)
    a, b = str(tmp_path / "a.miracle"), str(tmp_path / "b.miracle")
    model.code_image_greedy(None, img, 7, comp_file_path=a, **KW)
    model.code_image_greedy(None, img, 7, comp_file_path=b, **KW)
    assert open(a, "rb").read() == open(b, "rb").read()


def test_codec_with_empirical_dists_and_index_ac(P, tmp_path):
    """build_empirical_dists' count models drive the group-size coders, and
    with use_index_ac the importance indices go through the arithmetic coder."""
    model = _model(P, seed=3)
    imgs = [_image(64, 64, seed=s) for s in (3, 4)]
    kw = dict(KW)
    gs1, gs2, si1, si2 = P.build_empirical_dists(model, imgs, seed=11, **kw)
    assert gs1[0] == 2 and gs2[0] == 2 and si1[0] == 2 and si2[0] == 2
    assert gs2.size == 1 + 2 ** kw["second_level_max_group_size_bits"]
    path = str(tmp_path / "i.miracle")
    (s2, s1), _ = model.code_image_greedy(
        None, imgs[0], 11, comp_file_path=path, use_importance_sampling=True,
        first_level_group_dist_counts=gs1, second_level_group_dist_counts=gs2,
        use_index_ac=True, first_level_sample_ac=si1, second_level_sample_ac=si2, **kw)
    (t2, t1), _ = model.code_image_greedy(None, imgs[0], 11, comp_file_path=str(tmp_path / "j"),
                                          use_importance_sampling=True, **kw)
    _eq(s2, t2, "level-2 sample (index AC vs Elias-delta)")
    _eq(s1, t1, "level-1 sample (index AC vs Elias-delta)")
    rec = model.decode_image_greedy(None, path, use_importance_sampling=True,
                                    first_level_group_dist_counts=gs1,
                                    second_level_group_dist_counts=gs2, use_index_ac=True,
                                    first_level_sample_ac=si1, second_level_sample_ac=si2)
    rec2 = model.decode_image_greedy(None, str(tmp_path / "j"), use_importance_sampling=True,
                                     first_level_max_group_size_bits=4,
                                     second_level_max_group_size_bits=2)
    _eq(rec, rec2, "reconstruction (index AC vs Elias-delta)")


def test_return_flags(P):
    model = _model(P, seed=4)
    img = _image(64, 64, seed=5)
    gi2 = model.code_image_greedy(None, img, 3, return_second_level_group_sizes=True, **KW)
    assert gi2[0] == 0 and gi2[-1] == 8 * 1 * 1
    ind2 = model.code_image_greedy(None, img, 3, return_second_level_indices=True, **KW)
    assert len(ind2) == len(gi2) - 1 and min(ind2) >= 1
    gi1 = model.code_image_greedy(None, img, 3, return_first_level_group_sizes=True, **KW)
    assert gi1[0] == 0 and gi1[-1] == 32 * 4 * 4


def test_codec_rejects_grid_mismatch(P):
    """Sizes that are not multiples of 64: TF 'same' padding rounds the level-1
    grid up (100x150 -> 7x10) but SynthesisTransform_2 returns 4x the level-2
    grid (8x12); the reference fails combining them (pln.py:165-185), so does
    this codec, with a clear message."""
    model = _model(P, seed=6)
    with pytest.raises(ValueError, match="same shape"):
        model.code_image_greedy(None, _image(100, 150, seed=6), 5, **KW)


@pytest.mark.parametrize("hw,use_perm,level1", [((64, 320), False, "greedy"),
                                                 ((192, 64), False, "importance")])
def test_codec_no_permutation(P, oracle, tmp_path, hw, use_perm, level1):
    """use_permutation=False (identity permutation) round trips bit-exactly,
    on non-square grids."""
    model = _model(P, seed=6)
    img = _image(*hw, seed=6)
    path = str(tmp_path / "np.miracle")
    imp = level1 == "importance"
    (s2, s1), summ = model.code_image_greedy(None, img, 5, comp_file_path=path,
                                             use_permutation=use_perm,
                                             use_importance_sampling=imp, **KW)
    shape1 = tuple(model.latent_distributions(img, 5)["q1"].loc.shape)
    rec = model.decode_image_greedy(None, path, use_importance_sampling=imp,
                                    use_permutation=use_perm, first_level_max_group_size_bits=4,
                                    second_level_max_group_size_bits=2)
    assert rec.shape == (hw[0], hw[1], 3)
    if not imp:
        z1 = P.unpermute_unflatten(torch.from_numpy(s1).cuda(), None, shape1)
        with torch.no_grad():
            want = model.synthesis_transform_1(z1)[0].permute(1, 2, 0).cpu().numpy()
        _eq(rec, want, "reconstruction")
    else:
        assert np.isfinite(rec).all()
