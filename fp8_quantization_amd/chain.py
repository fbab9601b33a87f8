"""The word-image hand-off between consecutive approx convolutions (fp8a_conv2d_chain).

Every convolution on the matrix-core path (csrc/gemm_f8mx.h) reads its input A as one 32-bit word
per element, which its xm_decode_a pre-pass writes from the fp32 input (after the layer's fused
input quantizer): the pass reads x back and writes the image, 8 B of HBM traffic per element,
7.6 % of the ResNet-18 forward (profiles/rocprof_r18_e4m3_r3_breakdown.txt).  In the fixed-range
eval forward the convolution that PRODUCES x already holds every value in its store, so it
writes the next convolution's words there (fq_next(y) -> word, bit for bit the pre-pass's), and
the next launch runs its pre-pass gated: it only writes the input quantizer's bias, or re-decodes
x when an element left the window.  The reference has no counterpart (its operators materialise
im2col columns, approx_calculation.py:724-747); the per-layer op order of the reference
(hijacker.py:77-115, quantized_folded_bn.py:30-83) is unchanged.
"""
import os

# FP8A_CHAIN=0 keeps every convolution's own A operand pre-pass
CHAIN = os.environ.get("FP8A_CHAIN", "1") != "0"


class WordChain:
    """The word-image hand-off (fp8a_conv2d_chain, include/fp8approx.h) for one approx
    convolution of a fixed-range forward: ``in_image`` is its input's word image, emitted by the
    convolution that produced the input (used when this layer fuses its input quantizer), and
    ``next_layer`` the convolution that consumes its output, for which it emits one while storing
    (when that layer fuses its input quantizer and its launch would read an image).  After the
    launch, ``emitted`` is the image written for next_layer, or None -- the next layer gets an
    image only from a launch that wrote it, so a stale buffer is never read.  Results are bit for
    bit those of the unchained launches: the same words, the fp32 tensors still written."""

    def __init__(self, in_image=None, next_layer=None):
        self.in_image = in_image
        self.next_layer = next_layer
        self.emitted = None

    def request(self, layer, x, qin):
        """The ``chain`` argument of approx_conv2d for layer's launch on x, or None."""
        in_img = self.in_image if qin is not None else None
        out = None
        nxt = self.next_layer
        # (an ungrouped launch emits the E4M3 / E5M2 and table forms; a depthwise launch the matrix-core
        # form (1: the staged table-form kernel, round 6) or the v5 form (3: the staged v5 kernel) --
        # any other launch flags the image invalid)
        nq = nxt.chain_input_quantizer() if nxt is not None else None
        form = nxt.chain_wants_image() if nq is not None else 0
        if form and layer.groups != 1 and form not in (1, 3):
            form = 0
        if form:
            Bn, _, H, W = x.shape
            kh, kw = layer.kernel_size
            Ho = (H + 2 * layer.padding[0] - layer.dilation[0] * (kh - 1) - 1) // layer.stride[0] + 1
            Wo = (W + 2 * layer.padding[1] - layer.dilation[1] * (kw - 1) - 1) // layer.stride[1] + 1
            E, M, _, _ = nxt._approx_config()
            img = nxt.chain_image((Bn, layer.out_channels, Ho, Wo), x.device, form)
            nbR = nxt._default_bias(nxt.get_res_fp_bias(), E, x.device)
            out = (img, tuple(nxt.padding), (nq.maxval, nq.n_bits, nq._mbits_int, nq.sign_bits), nbR, M, form - 1)
        if in_img is None and out is None:
            return None
        return in_img, out

    def done(self, ch):
        self.emitted = ch[1][0] if ch[1] is not None else None


class ChainConsumerMixin:
    """What WordChain asks of a consumer convolution (mixed into the approx conv operators)."""

    def chain_input_quantizer(self):
        """The per-tensor input FPQuantizer this layer's next forward fuses into its launch, or None."""
        from .quantization.quantized_folded_bn import BNFusedHijacker
        if not CHAIN or not isinstance(self, BNFusedHijacker) or self._fused_epilogue() is None:
            return None
        return self._fused_input_quantizer(self._qa())

    def chain_wants_image(self):
        """The input word image this layer's launch would read: 0 none, 1 the matrix-core form, 2 the
        tensor-bias table form (single-output-channel groups), 3 the v5 matrix-core form
        (fp8a_conv2d_wants_image)."""
        # keyed on the layer's approx parameters and the library's option generation (an option such
        # as af32_maxct changes the answer), so the table is not rebuilt and re-listed every forward
        from . import _lib
        p = self.custom_approx_params
        key = (tuple(sorted((k, v) for k, v in p.items() if isinstance(v, (bool, int, float, str)))),
               _lib.option_generation())
        cached = getattr(self, "_chain_wants", None)
        if cached is None or cached[0] != key:
            from .approx_ops import conv2d_wants_image
            E, M, table, flags = self._approx_config()
            cached = (key, conv2d_wants_image(self.out_channels, self.kernel_size, self.padding, self.groups, E, M,
                                              table, flags, self.stride, self.dilation))
            self._chain_wants = cached
        return cached[1]

    def chain_image(self, in_shape, device, form=1):
        """This layer's input word image buffer (allocated and initialised once per shape): with
        this layer's padding as border (form 1), or none (form 2, the table form's plain words)."""
        pad = tuple(self.padding) if form != 2 else (0, 0)
        key = (tuple(in_shape), pad, str(device))
        cached = getattr(self, "_chain_img", None)
        if cached is None or cached[0] != key:
            from .approx_ops import new_word_image
            cached = (key, new_word_image(*in_shape, pad[0], pad[1], device))
            self._chain_img = cached
        return cached[1]
