"""fp8a_matmul_block (the fused linear launch of QCustomLinearTorch) against the separate passes
the reference runs (approx_calculation.py:1007-1023 and its ViT callers,
vit_quantized_approx.py:137-156): input fake-quant -> approx product -> ``out += bias`` ->
``+ residual`` -> output fake-quant.  Every case must be bit-identical to the unfused sequence
of this library's own ops (each of which is pinned to the oracle elsewhere), and the quantizer
biases it reports must equal the ones the quantizers compute."""
import numpy as np
import pytest
import torch

from fp8_quantization_amd import approx_ops as ao
from fp8_quantization_amd.error_tables import get_error_table_NN

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _native():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from fp8_quantization_amd import _lib
    _lib.load()


def _operands(Mr, K, N, E, M, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn((Mr, K), generator=g).to(DEV)
    w = (torch.randn((N, K), generator=g) * 0.05).to(DEV)
    mxw = w.abs().amax(dim=1)
    wq, bw = ao.fp8_fake_quantize(w, mxw, 8, M, per_row=True)
    bias = (torch.randn(N, generator=g) * 0.1).to(DEV)
    res = torch.randn((Mr, N), generator=g).to(DEV)
    return x, wq, bw, bias, res


def _bits(t):
    return t.detach().cpu().numpy().view(np.uint32)


CASES = [  # (M rows, K, N, E, M, with qin, with post)
    (300, 192, 160, 4, 3, False, False),
    (300, 192, 160, 4, 3, True, False),
    (257, 768, 96, 4, 3, True, True),
    (64, 4096, 128, 4, 3, True, True),     # split-K
    (200, 256, 64, 3, 4, True, True),      # E3M4: materialized input quantization, tile-table kernel
    (130, 96, 72, 2, 5, False, True),      # E2M5
    (96, 160, 64, 4, 3, True, True, 1),    # bR = 1: terms beyond the e4m3 range -> gated exact kernel with qin
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}x{c[1]}x{c[2]}-E{c[3]}M{c[4]}-q{int(c[5])}p{int(c[6])}"
                                             + (f"-bR{c[7]}" if len(c) > 7 else "") for c in CASES])
def test_matmul_block_equals_separate_passes(case):
    Mr, K, N, E, M, with_qin, with_post = case[:7]
    x, wq, bw, bias, res = _operands(Mr, K, N, E, M, seed=Mr + K + N)
    table = get_error_table_NN(E, M, withComp=False, dnsmp_factor=3)
    flags = ao.make_flags(with_approx=True, with_s2nn2s_opt=True, quant_btw_mult_accu=True)
    in_mx = x.abs().amax().reshape(1)
    xq, bx = ao.fp8_fake_quantize(x, in_mx, 8, M)
    out_mx = torch.tensor([7.5], device=DEV)
    bR = case[7] if len(case) > 7 else 2 ** (E - 1) + 3

    # reference order, one pass each
    ref = ao.approx_matmul(xq, wq.t(), E, M, bx, bw, bR, table, flags=flags)
    ref = ref + bias
    if with_post:
        ref, bo = ao.fp8_fake_quantize(ref + res, out_mx, 8, M)

    qin = (in_mx, 8, M, 1) if with_qin else None
    post = (res, 0, 0.0, 0.0, (out_mx, 8, M, 1)) if with_post else None
    got, ib, ob = ao.approx_matmul_block(x if with_qin else xq, wq.t(), E, M, None if with_qin else bx, bw, bR,
                                         table, flags=flags, bias=bias, qin=qin, post=post)
    assert np.array_equal(_bits(got), _bits(ref)), np.abs(got - ref).max().item()
    if with_qin:
        assert ib.item() == bx.reshape(-1)[0].item()
    if with_post:
        assert ob.item() == bo.reshape(-1)[0].item()


def test_matmul_block_rejects_bad_residual():
    x, wq, bw, bias, res = _operands(16, 32, 8, 4, 3, seed=1)
    flags = ao.make_flags(with_approx=True, with_s2nn2s_opt=True, quant_btw_mult_accu=True)
    with pytest.raises(AssertionError):
        ao.approx_matmul_block(x, wq.t(), 4, 3, 12, bw, 15, None, flags=flags,
                               post=(res[:, :4], 0, 0.0, 0.0, None))


@pytest.mark.parametrize("version", [9, 5])
def test_linear_operator_fixed_range_forward(version):
    """QCustomLinearTorch in the fixed-range approx forward (input quantizer and bias fused into
    the launch for v9; v5 keeps its own path) equals the explicit sequence: quantize the input,
    approx_multiply, + bias."""
    from fp8_quantization_amd.approx_calculation import QCustomLinearTorch
    from fp8_quantization_amd.resnet_workload import approx_qparams
    qp = approx_qparams(expo_width=4, mant_width=3) if version == 9 else \
        approx_qparams(expo_width=3, mant_width=4, withComp=True)
    if version == 5:
        qp["custom_approx_params"].update(approx_version=5, sim_hw_add_OFUF=True)
    torch.manual_seed(2)
    m = QCustomLinearTorch(in_features=48, out_features=24, bias=True, **qp).to(DEV).eval()
    x = torch.randn(10, 48, device=DEV)
    with torch.no_grad():
        m.quantized()
        m.estimate_ranges()
        m(x)
        m.fix_ranges()
        got = m(x)
        xq = m.activation_quantizer(x)
        wq, b = m.get_params()
        ref = m.approx_multiply(xq, wq.t(), m.get_acts_fp_bias(), m.get_weights_fp_bias(), m.get_res_fp_bias()) + b
    assert np.array_equal(_bits(got), _bits(ref))


GELU_CASES = [  # (M rows, K, N, E, M, with output quantizer)
    (300, 192, 160, 4, 3, True),
    (257, 768, 320, 4, 3, False),
    (64, 4096, 128, 4, 3, True),     # split-K: the GELU tail in the reduction
    (200, 256, 64, 3, 4, True),      # E3M4 tile-table kernel
    (130, 96, 72, 2, 5, True),       # E2M5
    (96, 160, 64, 4, 3, True, 1),    # bR = 1: the gated exact kernel's store
]


@pytest.mark.parametrize("case", GELU_CASES, ids=[f"{c[0]}x{c[1]}x{c[2]}-E{c[3]}M{c[4]}-q{int(c[5])}"
                                                   + (f"-bR{c[6]}" if len(c) > 6 else "") for c in GELU_CASES])
def test_matmul_block_gelu_tail_equals_torch_gelu(case):
    """post_act 2: fq_out(gelu(fq_in(A) @ B + bias)) in one launch, bit-identical to the product,
    then torch's nn.GELU() (the reference's intermediate_act_fn), then the output fake-quant --
    vit_quantized_approx.py:117-135."""
    Mr, K, N, E, M, with_q = case[:6]
    x, wq, bw, bias, _ = _operands(Mr, K, N, E, M, seed=Mr * 3 + K + N)
    table = get_error_table_NN(E, M, withComp=False, dnsmp_factor=3)
    flags = ao.make_flags(with_approx=True, with_s2nn2s_opt=True, quant_btw_mult_accu=True)
    in_mx = x.abs().amax().reshape(1)
    xq, bx = ao.fp8_fake_quantize(x, in_mx, 8, M)
    out_mx = torch.tensor([3.25], device=DEV)
    bR = case[6] if len(case) > 6 else 2 ** (E - 1) + 3
    ref = torch.nn.GELU()(ao.approx_matmul(xq, wq.t(), E, M, bx, bw, bR, table, flags=flags) + bias)
    if with_q:
        ref, bo = ao.fp8_fake_quantize(ref, out_mx, 8, M)
    post = (None, 2, 0.0, 0.0, (out_mx, 8, M, 1) if with_q else None)
    got, ib, ob = ao.approx_matmul_block(x, wq.t(), E, M, None, bw, bR, table, flags=flags, bias=bias,
                                         qin=(in_mx, 8, M, 1), post=post)
    assert np.array_equal(_bits(got), _bits(ref)), np.abs(got - ref).max().item()
    if with_q:
        assert ob.item() == bo.reshape(-1)[0].item()


def test_conv_block_rejects_gelu_tail():
    from fp8_quantization_amd import _lib
    L = _lib.load()
    x = torch.zeros((1, 4, 4, 4), device=DEV)
    w = torch.zeros((4, 4, 1, 1), device=DEV)
    y = torch.empty_like(x)
    b = torch.zeros(4, dtype=torch.int32, device=DEV)
    tab = torch.zeros((8, 8), dtype=torch.int32)
    ws = torch.zeros(1 << 16, dtype=torch.uint8, device=DEV)
    rc = L.fp8a_conv2d_block(_lib.dev_ptr(x), _lib.dev_ptr(w), _lib.dev_ptr(y), 1, 4, 4, 4, 4, 1, 1, 1, 1, 0, 0, 1, 1, 1,
                             4, 3, _lib.dev_ptr(b), _lib.dev_ptr(b), _lib.dev_ptr(b), _lib.host_ptr(tab), 0, None, 0, 0.0,
                             0.0, None, 0, 0, 0, None, None, None, 2, 0.0, 0.0, None, 0, 0, 0, None, None,
                             _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(DEV))
    assert rc == -1
