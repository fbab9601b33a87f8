"""The word-image hand-off between consecutive approx convolutions (fp8a_conv2d_chain, round 4).

A producer convolution writes, next to its fp32 output y, the consumer's A operand word image
(the words of fq_next(y)); the consumer's launch then runs its A pre-pass gated.  Checked:
  * op level, bit-identical consumer outputs and input-quantizer biases with and without the
    image: plain producer store, BN + ReLU epilogue, a residual tail with an output quantizer,
    a split-K producer (the reduction emits), a producer whose gated exact kernel recomputes
    units (the exact kernel emits), E4M3 and E5M2;
  * an image flagged invalid is re-decoded from y (same result);
  * a producer that cannot emit (grouped) flags the image invalid; a tensor-bias depthwise producer
    (the staged table-form kernel) emits the next 1x1 convolution's matrix-core words (round 6);
  * model level: ResNet-18 / ResNet-50 logits bit-identical with the hand-off on and off, and the
    hand-off really ran (fewer full pre-passes: counted through the launch trace of a profiler-free
    counter, the consumer launches that read an image).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _native():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from fp8_quantization_amd import _lib
    _lib.load()


def _grid(g, shape, M, lo=-6, hi=3, zero=0.3):
    e = torch.randint(lo, hi, shape, generator=g).float()
    m = torch.randint(0, 2 ** M, shape, generator=g).float()
    v = torch.ldexp(1.0 + m / 2 ** M, e.int()) * (torch.randint(0, 2, shape, generator=g).float() * 2 - 1)
    v[torch.rand(shape, generator=g) < zero] = 0.0
    return v


def _bits(t):
    return t.detach().cpu().contiguous().view(torch.int32)


def _run_pair(E, M, cin, cmid, cout, hw, Bn, k1, k2, p1, p2, epilogue, post, seed, bad_w=False, fmt_table=None):
    """producer conv1 (x -> y) and consumer conv2 (y -> z, fused input quantizer), unchained and
    chained; returns (z, z_chained, consumer input bias pair)."""
    from fp8_quantization_amd.approx_ops import approx_conv2d, make_flags, new_word_image, bn_act_epilogue
    from fp8_quantization_amd.error_tables import get_error_table_NN
    g = torch.Generator().manual_seed(seed)
    tab = fmt_table if fmt_table is not None else get_error_table_NN(E, M, False, 3, zero_table_ext=(E, M) == (5, 2))
    fl = make_flags(True, True, True)
    b = 2 ** (E - 1)
    x = _grid(g, (Bn, cin, hw, hw), M).to(DEV)
    w1 = _grid(g, (cmid, cin, k1, k1), M, -8, 0, 0.0).to(DEV)
    w2 = _grid(g, (cout, cmid, k2, k2), M, -8, 0, 0.0).to(DEV)
    if bad_w:  # off-grid weights: the producer's gated exact kernel recomputes their column units
        w1[3, 0, 0, 0] = 0.3333
    bA, bR1, bR2 = b + 2, b + 1, b
    bW1 = torch.full((cmid,), b + 6, dtype=torch.int32, device=DEV)
    bW2 = torch.full((cout,), b + 6, dtype=torch.int32, device=DEV)
    ep = None
    if epilogue:
        gam = torch.rand(cmid, generator=g) + 0.5
        ep = bn_act_epilogue(torch.randn(cmid, generator=g) * 0.1, torch.rand(cmid, generator=g) + 0.5, gam,
                             torch.randn(cmid, generator=g) * 0.1, 1e-5, torch.nn.ReLU())
        ep = (ep[0].to(DEV),) + tuple(ep[1:])
    mx_out = torch.tensor([6.0], device=DEV)
    pst = None
    if post:
        res = _grid(g, (Bn, cmid, hw, hw), M).to(DEV)
        pst = (res, 1, 0.0, float("inf"), (mx_out, 8, M, 1))
    mx2 = torch.tensor([5.5], device=DEV)
    qin2 = (mx2, 8, M, 1)
    bR2t = torch.tensor([bR2], dtype=torch.int32, device=DEV)
    args1 = dict(flags=fl, padding=(p1, p1), epilogue=ep)
    args2 = dict(flags=fl, padding=(p2, p2))

    def produce(chain=None):
        kw = dict(args1)
        if pst is not None:
            kw["post"] = pst
        if chain is not None or pst is not None:
            out = approx_conv2d(x, w1, E, M, bA, bW1, bR1, tab, chain=chain, **kw)
            return out[0]
        return approx_conv2d(x, w1, E, M, bA, bW1, bR1, tab, **kw)

    y = produce()
    z, ib, _ = approx_conv2d(y, w2, E, M, None, bW2, bR2t, tab, qin=qin2, **args2)
    img = new_word_image(Bn, cmid, hw, hw, p2, p2, DEV)
    y2 = produce(chain=(None, (img, (p2, p2), qin2, bR2t, M)))
    assert torch.equal(_bits(y), _bits(y2)), "producer output changed by the emission"
    z2, ib2, _ = approx_conv2d(y2, w2, E, M, None, bW2, bR2t, tab, qin=qin2, chain=(img, None), **args2)
    torch.cuda.synchronize()
    header = int(img[:4].view(torch.int32).item())
    return z, z2, (ib, ib2), header, (y2, w2, bW2, bR2t, qin2, args2, img, tab)


@pytest.mark.parametrize("E,M", [(4, 3), (5, 2)])
@pytest.mark.parametrize("case", ["plain", "bn_relu", "tail", "splitk", "fallback"])
def test_chain_bit_identical(E, M, case):
    from fp8_quantization_amd import _lib
    kw = dict(cin=16, cmid=64, cout=64, hw=14, Bn=3, k1=3, k2=3, p1=1, p2=1, epilogue=False, post=False, seed=7)
    if case == "bn_relu":
        kw.update(epilogue=True)
    elif case == "tail":
        kw.update(epilogue=True, post=True)
    elif case == "splitk":  # long K, few output tiles: split-K (the reduction kernel stores y)
        kw.update(cin=512, cmid=128, cout=64, hw=7, Bn=2, seed=8)
    elif case == "fallback":
        kw.update(bad_w=True, seed=9)
    _lib.fallback_stats(reset=True)
    z, z2, (ib, ib2), header, _ = _run_pair(E, M, **kw)
    assert header == 0, "the emitted image was flagged invalid"
    assert torch.equal(_bits(z), _bits(z2)), "consumer output differs with the word image"
    assert torch.equal(ib, ib2)
    if case == "fallback":
        assert _lib.fallback_stats()["exact_launches"] >= 1


def test_invalid_image_is_redecoded():
    from fp8_quantization_amd.approx_ops import approx_conv2d
    z, _, _, _, (y2, w2, bW2, bR2t, qin2, args2, img, tab) = _run_pair(
        4, 3, cin=16, cmid=64, cout=64, hw=14, Bn=2, k1=3, k2=3, p1=1, p2=1, epilogue=True, post=False, seed=11)
    img[4:].zero_()  # garbage words ...
    img[:4].view(torch.int32).fill_(1)  # ... flagged invalid: the gated pre-pass re-decodes y
    z3, _, _ = approx_conv2d(y2, w2, 4, 3, None, bW2, bR2t, tab, qin=qin2, chain=(img, None), **args2)
    assert torch.equal(_bits(z), _bits(z3))


def test_grouped_producer_flags_invalid():
    from fp8_quantization_amd.approx_ops import approx_conv2d, make_flags, new_word_image
    from fp8_quantization_amd.error_tables import get_error_table_NN
    g = torch.Generator().manual_seed(3)
    x = _grid(g, (2, 8, 10, 10), 3).to(DEV)
    w = _grid(g, (8, 4, 3, 3), 3, -8, 0, 0.0).to(DEV)
    img = new_word_image(2, 8, 10, 10, 1, 1, DEV)
    tab = get_error_table_NN(4, 3, False, 3)
    approx_conv2d(x, w, 4, 3, 10, torch.full((8,), 14, dtype=torch.int32, device=DEV), 9, tab,
                  flags=make_flags(True, True, True), padding=(1, 1), groups=2,
                  chain=(None, (img, (1, 1), (torch.tensor([4.0], device=DEV), 8, 3, 1),
                                torch.tensor([8], dtype=torch.int32, device=DEV), 3)))
    torch.cuda.synchronize()
    assert int(img[:4].view(torch.int32).item()) != 0


def test_v5_producer_flags_invalid():
    """A producer on the v5 matrix-core form (gemm_v5mx_kernel, whose store does not emit) feeding
    a v9 E5M2 consumer: the image comes back flagged invalid and the consumer, which then
    re-decodes y, gives the unchained result."""
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_ops import approx_conv2d, make_flags, make_flags_v5, new_word_image
    from fp8_quantization_amd.error_tables import get_error_table_NN
    g = torch.Generator().manual_seed(5)
    x = _grid(g, (2, 16, 10, 10), 2).to(DEV)
    w1 = _grid(g, (32, 16, 3, 3), 2, -8, 0, 0.0).to(DEV)
    w2 = _grid(g, (32, 32, 3, 3), 2, -8, 0, 0.0).to(DEV)
    zero = torch.zeros((4, 4), dtype=torch.int32)
    tab = get_error_table_NN(5, 2, False, 3, zero_table_ext=True)
    bW = torch.full((32,), 22, dtype=torch.int32, device=DEV)
    qin2 = (torch.tensor([5.5], device=DEV), 8, 2, 1)
    bR2 = torch.tensor([16], dtype=torch.int32, device=DEV)
    img = new_word_image(2, 32, 10, 10, 1, 1, DEV)
    _lib.path_stats(reset=True)
    out = approx_conv2d(x, w1, 5, 2, 18, bW, 14, zero, flags=make_flags_v5(True, True, True), padding=(1, 1),
                        chain=(None, (img, (1, 1), qin2, bR2, 2)))
    y = out[0]
    assert _lib.path_stats(reset=True)["v5mx"] >= 1
    torch.cuda.synchronize()
    assert int(img[:4].view(torch.int32).item()) != 0
    args2 = dict(flags=make_flags(True, True, True), padding=(1, 1))
    z, _, _ = approx_conv2d(y, w2, 5, 2, None, bW, bR2, tab, qin=qin2, **args2)
    z2, _, _ = approx_conv2d(y, w2, 5, 2, None, bW, bR2, tab, qin=qin2, chain=(img, None), **args2)
    assert torch.equal(_bits(z), _bits(z2))


@pytest.mark.parametrize("arch,fmt", [("resnet18", (4, 3)), ("resnet50", (4, 3)), ("resnet18", (5, 2))])
def test_model_logits_identical_with_chain(arch, fmt, monkeypatch):
    from fp8_quantization_amd import chain, resnet_workload as rw
    E, M = fmt
    torch.manual_seed(1)
    m = getattr(rw, arch + "_approx")(bn_stats_batches=2, device=DEV, expo_width=E, mant_width=M).to(DEV).eval()
    g = torch.Generator().manual_seed(2)
    m.quantized()
    m.estimate_ranges()
    with torch.no_grad():
        m(torch.randn((4, 3, 64, 64), generator=g).to(DEV))
    m.fix_ranges()
    x = torch.randn((3, 3, 64, 64), generator=g).to(DEV)
    emitted = []
    orig_done = chain.WordChain.done

    def done(self, ch):
        orig_done(self, ch)
        emitted.append(self.emitted is not None)
    monkeypatch.setattr(chain.WordChain, "done", done)
    with torch.no_grad():
        on = m(x)
    assert sum(emitted) >= (7 if arch == "resnet18" else 10), emitted  # the hand-off ran
    monkeypatch.setattr(chain, "CHAIN", False)
    with torch.no_grad():
        off = m(x)
    assert torch.equal(_bits(on), _bits(off)), "logits differ with the word-image hand-off"


@pytest.mark.parametrize("E,M", [(4, 3), (5, 2)])
@pytest.mark.parametrize("stride", [1, 2])
def test_table_form_handoff_to_depthwise(E, M, stride):
    """next_form 1: the producer emits the tensor-bias table form's words (no border) for a
    depthwise consumer that fuses its input quantizer; the consumer's tbx pre-pass runs gated.
    Consumer outputs and its input-quantizer bias bit-identical to the unchained pair (the
    automatic use in models is opt-in, FP8A_CHAIN_TBX=1: DESIGN.md §3i)."""
    from fp8_quantization_amd.approx_ops import approx_conv2d, make_flags, new_word_image
    from fp8_quantization_amd.error_tables import get_error_table_NN
    g = torch.Generator().manual_seed(11 + stride + M)
    tab = get_error_table_NN(E, M, False, 3, zero_table_ext=(E, M) == (5, 2))
    fl = make_flags(True, True, True)
    b = 2 ** (E - 1)
    Bn, cin, cmid, hw = 2, 16, 48, 14
    x = _grid(g, (Bn, cin, hw, hw), M).to(DEV)
    w1 = _grid(g, (cmid, cin, 1, 1), M, -8, 0, 0.0).to(DEV)
    w2 = _grid(g, (cmid, 1, 3, 3), M, -8, 0, 0.0).to(DEV)
    bA, bR1 = b + 2, b + 1
    bW1 = torch.full((cmid,), b + 6, dtype=torch.int32, device=DEV)
    bW2 = torch.full((cmid,), b + 6, dtype=torch.int32, device=DEV)
    bR2 = torch.tensor([b], dtype=torch.int32, device=DEV)
    qin2 = (torch.tensor([5.5], device=DEV), 8, M, 1)
    args2 = dict(flags=fl, padding=(1, 1), stride=(stride, stride), groups=cmid)
    y = approx_conv2d(x, w1, E, M, bA, bW1, bR1, tab, flags=fl)
    z, ib, _ = approx_conv2d(y, w2, E, M, None, bW2, bR2, tab, qin=qin2, **args2)
    img = new_word_image(Bn, cmid, hw, hw, 0, 0, DEV)
    y2 = approx_conv2d(x, w1, E, M, bA, bW1, bR1, tab, flags=fl,
                       chain=(None, (img, (1, 1), qin2, bR2, M, 1)))[0]
    assert torch.equal(_bits(y), _bits(y2)), "producer output changed by the emission"
    z2, ib2, _ = approx_conv2d(y2, w2, E, M, None, bW2, bR2, tab, qin=qin2, chain=(img, None), **args2)
    torch.cuda.synchronize()
    assert int(img[:4].view(torch.int32).item()) == 0, "the emitted image was flagged invalid"
    assert torch.equal(_bits(z), _bits(z2)) and torch.equal(ib, ib2)


@pytest.mark.parametrize("stride", [1, 2])
def test_v5_depthwise_handoff_to_v5_gemm(stride):
    """A v5 depthwise layer (the staged conv_v5ds_kernel) emitting the v5 matrix-core words of the
    next 1x1 convolution's input (fp8a_conv2d_chain next_form 2): the image stays valid, and the
    consumer reading it gives the unchained result bit for bit, with the same input-quantizer bias."""
    from fp8_quantization_amd.approx_ops import approx_conv2d, make_flags_v5, new_word_image
    g = torch.Generator().manual_seed(7 + stride)
    C, H = 24, 15
    x = _grid(g, (2, C, H, H), 2).to(DEV)
    wd = _grid(g, (C, 1, 3, 3), 2, -8, 0, 0.0).to(DEV)
    wp = _grid(g, (40, C, 1, 1), 2, -8, 0, 0.0).to(DEV)
    tab = torch.as_tensor(np.array([[0, -1, 2, 0], [1, 0, -2, 1], [0, 3, 0, -1], [-3, 1, 1, 0]], np.int32))
    fl = make_flags_v5(True, True, True)
    bWd = torch.full((C,), 18, dtype=torch.int32, device=DEV)
    bWp = torch.full((40,), 20, dtype=torch.int32, device=DEV)
    bR = torch.tensor([12], dtype=torch.int32, device=DEV)
    qin1 = (torch.tensor([9.0], device=DEV), 8, 2, 1)
    qin2 = (torch.tensor([3.5], device=DEV), 8, 2, 1)
    Ho = (H + 2 - 3) // stride + 1
    img = new_word_image(2, C, Ho, Ho, 0, 0, DEV)
    args1 = dict(flags=fl, stride=(stride, stride), padding=(1, 1), groups=C)
    y, _, _ = approx_conv2d(x, wd, 5, 2, None, bWd, bR, tab, qin=qin1, chain=(None, (img, (0, 0), qin2, bR, 2, 2)),
                            **args1)
    y0, _, _ = approx_conv2d(x, wd, 5, 2, None, bWd, bR, tab, qin=qin1, **args1)
    torch.cuda.synchronize()
    assert torch.equal(_bits(y), _bits(y0))
    assert int(img[:4].view(torch.int32).item()) == 0, "the staged v5 depthwise producer did not emit"
    z, ib, _ = approx_conv2d(y, wp, 5, 2, None, bWp, bR, tab, qin=qin2, flags=fl)
    z2, ib2, _ = approx_conv2d(y, wp, 5, 2, None, bWp, bR, tab, qin=qin2, flags=fl, chain=(img, None))
    assert torch.equal(_bits(z), _bits(z2)) and torch.equal(ib, ib2)


def test_mobilenet_v5_logits_identical_with_chain(monkeypatch):
    """BASELINE config 3's v5 mode (MobileNetV2 E5M2, approx_version 5 with the OF / UF switches):
    logits with the depthwise -> projection hand-off on and off, to the bit."""
    from fp8_quantization_amd import chain
    from fp8_quantization_amd.mobilenet_workload import mobilenet_v2_approx
    torch.manual_seed(3)
    m = mobilenet_v2_approx(input_size=64, n_class=100, bn_stats_batches=1, device=DEV, expo_width=5, mant_width=2,
                            dnsmp_factor=3, with_approx=True, with_s2nn2s_opt=True, quant_btw_mult_accu=True,
                            approx_version=5, withComp=True, sim_hw_add_OFUF=True, with_OF_opt=True,
                            with_UF_opt=True).to(DEV).eval()
    g = torch.Generator().manual_seed(4)
    m.quantized()
    m.estimate_ranges()
    with torch.no_grad():
        m(torch.randn((2, 3, 64, 64), generator=g).to(DEV))
    m.fix_ranges()
    x = torch.randn((3, 3, 64, 64), generator=g).to(DEV)
    emitted = []
    orig_done = chain.WordChain.done

    def done(self, ch):
        orig_done(self, ch)
        emitted.append(self.emitted is not None)
    monkeypatch.setattr(chain.WordChain, "done", done)
    with torch.no_grad():
        on = m(x)
    assert sum(emitted) >= 10, emitted  # the depthwise layers emitted
    monkeypatch.setattr(chain, "CHAIN", False)
    with torch.no_grad():
        off = m(x)
    assert torch.equal(_bits(on), _bits(off)), "logits differ with the v5 word-image hand-off"


@pytest.mark.parametrize("E,M", [(4, 3), (5, 2)])
@pytest.mark.parametrize("stride", [1, 2])
def test_depthwise_handoff_to_matrix_core(E, M, stride):
    """A tensor-bias depthwise layer (the staged table-form conv_tbsg_kernel) emitting the matrix-core
    words of the next 1x1 convolution's input (fp8a_conv2d_chain next_form 0, round 6): its own output
    unchanged, the image valid, and the consumer reading it gives the unchained result bit for bit,
    with the same input-quantizer bias."""
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_ops import approx_conv2d, make_flags, new_word_image
    from fp8_quantization_amd.error_tables import get_error_table_NN
    g = torch.Generator().manual_seed(17 + stride + M)
    C, H = 24, 15
    b = 2 ** (E - 1)
    x = _grid(g, (2, C, H, H), M).to(DEV)
    wd = _grid(g, (C, 1, 3, 3), M, -8, 0, 0.0).to(DEV)
    wp = _grid(g, (40, C, 1, 1), M, -8, 0, 0.0).to(DEV)
    tab = get_error_table_NN(E, M, False, 3, zero_table_ext=(E, M) == (5, 2))
    fl = make_flags(True, True, True)
    bWd = torch.full((C,), b + 6, dtype=torch.int32, device=DEV)
    bWp = torch.full((40,), b + 6, dtype=torch.int32, device=DEV)
    bR = torch.tensor([b], dtype=torch.int32, device=DEV)
    qin1 = (torch.tensor([9.0], device=DEV), 8, M, 1)
    qin2 = (torch.tensor([3.5], device=DEV), 8, M, 1)
    Ho = (H + 2 - 3) // stride + 1
    img = new_word_image(2, C, Ho, Ho, 0, 0, DEV)
    args1 = dict(flags=fl, stride=(stride, stride), padding=(1, 1), groups=C)
    y, _, _ = approx_conv2d(x, wd, E, M, None, bWd, bR, tab, qin=qin1, chain=(None, (img, (0, 0), qin2, bR, M)),
                            **args1)
    y0, _, _ = approx_conv2d(x, wd, E, M, None, bWd, bR, tab, qin=qin1, **args1)
    torch.cuda.synchronize()
    assert torch.equal(_bits(y), _bits(y0))
    assert int(img[:4].view(torch.int32).item()) == 0, "the staged depthwise producer did not emit"
    _lib.path_stats(reset=True)
    z, ib, _ = approx_conv2d(y, wp, E, M, None, bWp, bR, tab, qin=qin2, flags=fl)
    z2, ib2, _ = approx_conv2d(y, wp, E, M, None, bWp, bR, tab, qin=qin2, flags=fl, chain=(img, None))
    assert _lib.path_stats(reset=True)["f8mx"] >= 2
    assert torch.equal(_bits(z), _bits(z2)) and torch.equal(ib, ib2)


@pytest.mark.parametrize("fmt", [(4, 3), (5, 2)])
def test_mobilenet_v9_logits_identical_with_chain(fmt, monkeypatch):
    """MobileNetV2 approx_v9 (E4M3, and config 3's E5M2): logits with every hand-off -- now also
    depthwise -> projection on the matrix-core words -- on and off, to the bit."""
    from fp8_quantization_amd import chain
    from fp8_quantization_amd.mobilenet_workload import mobilenet_v2_approx
    E, M = fmt
    torch.manual_seed(5)
    m = mobilenet_v2_approx(input_size=64, n_class=100, bn_stats_batches=1, device=DEV, expo_width=E,
                            mant_width=M).to(DEV).eval()
    g = torch.Generator().manual_seed(6)
    m.quantized()
    m.estimate_ranges()
    with torch.no_grad():
        m(torch.randn((2, 3, 64, 64), generator=g).to(DEV))
    m.fix_ranges()
    x = torch.randn((3, 3, 64, 64), generator=g).to(DEV)
    emitted = []
    orig_done = chain.WordChain.done

    def done(self, ch):
        orig_done(self, ch)
        emitted.append(self.emitted is not None)
    monkeypatch.setattr(chain.WordChain, "done", done)
    with torch.no_grad():
        on = m(x)
    assert sum(emitted) >= 15, emitted  # within and across the blocks, depthwise producers included
    monkeypatch.setattr(chain, "CHAIN", False)
    with torch.no_grad():
        off = m(x)
    assert torch.equal(_bits(on), _bits(off)), "logits differ with the word-image hand-off"
