/*
 * fp8approx.h -- C-ABI of the MI355X (gfx950) approx-FP8 matmul/conv engine.
 *
 * Drop-in boundary for the approx_v9 hot path of revollllt/FP8_quantization @ 2024-11-08.
 * Plain pointers and sizes only; every entry point is asynchronous on the given HIP stream,
 * allocates nothing and never synchronises the host (biases are DEVICE int32 scalars/arrays, so
 * a whole forward needs no .item() round trip -- unlike approx_calculation.py:780).
 *
 * Return codes: 0 ok; FP8A_EINVAL (shape/stride contract broken: the reference's
 * AssertionError, approx_matmul_whole_v9.py:20); FP8A_EFORMAT (unsupported (E, M): the
 * reference's ValueError, approx_matmul_whole_v9.py:590); FP8A_EHIP (HIP launch failure).
 * fp8a_last_error() gives a message for the last failure on the calling thread.
 *
 * Flags (same bit values the oracle uses):
 */
#ifndef FP8APPROX_H
#define FP8APPROX_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FP8A_APPROX 1u  /* with_approx: subtract the error table            v9:178-184 */
#define FP8A_S2N    2u  /* with_s2nn2s_opt: subnormal scale-up / scale-back v9:51-81   */
#define FP8A_QBMA   4u  /* quant_btw_mult_accu: Q_R before and after mult    v9:35,107 */
#define FP8A_GCLIP  8u  /* golden_clip_OF: Q_R clips overflow to max_norm   v9:283-286 */
#define FP8A_TB     16u /* biases are int tensors (single-column call): quirk F5,
                           approx_calculation.py:800-809 / v9:202                      */
/* The superseded integer-adder model (approx_matmul_whole_v5.py:10-183), opt-in: the term is
 * the sum of the operands' (expo << M | mant) codes minus (bA + bB - bR) << M plus the
 * compensation table entry (v5 tables, added), decoded with bR and signed.  The table argument
 * is then the v5 compensation table.  v9 accepts but ignores the OF/UF switches;
 * here they act as in v5 (approx_mult_new, v5:155-183). */
#define FP8A_V5     32u  /* use the v5 model                                    v5:10-183 */
#define FP8A_OFUF   64u  /* sim_hw_add_OFUF: wrap the code sum mod 2^(E+M)      v5:165-171 */
#define FP8A_OF_OPT 128u /* with_OF_opt: overflow -> max_norm_int               v5:173-174 */
#define FP8A_UF_OPT 256u /* with_UF_opt: underflow -> (sum mod 2^M)             v5:176-177 */

#define FP8A_OK       0
#define FP8A_EINVAL  -1
#define FP8A_EFORMAT -2
#define FP8A_EHIP    -3

typedef void *fp8a_stream_t; /* a hipStream_t (NULL = default stream) */

/* Library identification, e.g. "fp8approx gfx950 r1". */
const char *fp8a_version(void);
/* Message describing the last non-zero return on this thread ("" if none). */
const char *fp8a_last_error(void);

/*
 * Fallback counters of the library since it was loaded (or last reset), out[4]:
 *   [0] launches whose gated exact kernel ran (an operand off its FP8 grid or outside the fast
 *       path's exactness window, a bias outside the window, or a term beyond the e4m3 range),
 *   [1] 64 x 64 output units that kernel recomputed (only the marked units are: an off-grid A
 *       row marks its row units, a B column its column unit, a tile's out-of-range term its
 *       own units; a bias outside the window marks them all),
 *   [2] launches rerun in gemm_tt_kernel's f32 form (E3M4 left gemm_tt16_kernel's f16 window),
 *   [3] tensor-bias (depthwise) launches recomputed by the literal restatement.
 * Synchronises the device (diagnostics / benchmark reporting, not for the hot path); reset != 0
 * zeroes the counters after reading.
 */
int fp8a_fallback_stats(uint64_t *out, int reset);

/*
 * Launch paths the GEMM entry points took since load (host-side counters, no device sync), out[7]:
 *   [0] E4M3 / E5M2 per-pair matrix-core kernel (gemm_f8mx.h), [1] gemm_tt_kernel (E3M4 / E2M5),
 *   [2] gemm_tt16_kernel (E3M4), [3] gemm_fast_kernel (VALU tiled), [4] the exact kernel alone
 *   (tensor-bias products), [5] the dense exact product (fp8a_dense_*), [6] the v5 matrix-core
 *   form (gemm_v5mx.h).  reset != 0 zeroes them after reading.
 */
int fp8a_path_stats(uint64_t *out, int reset);

/*
 * Diagnostics: the byte size of one slot of the flag arena of (current device, stream), 0 before
 * the stream's first eager launch.  Slots only grow (a launch that needs more allocates a larger
 * arena; the old one is retired, never freed, so launches still in flight keep valid memory).
 */
size_t fp8a_flag_arena_slot_bytes(fp8a_stream_t stream);

/*
 * Kernel timing for benchmarks: while enabled (fp8a_kernel_timing(1); returns the previous
 * state), every GEMM records HIP events on its stream around its product kernel launch(es) only
 * (not its operand pre-passes, split-K reduction or gated exact kernel).  fp8a_kernel_time
 * synchronises on the recorded events and writes, per launch path in fp8a_path_stats order,
 * out[4 * path + 0..3] = (summed kernel milliseconds, launches, kernel dispatches, approx-MACs
 * M * N * K -- for the dense path, whose exact-product GEMM launches (dn_gemm*) are recorded too:
 * their algorithmic bytes, fp32 A read + fp32 C written + the packed B image read); reset != 0
 * forgets the recorded launches.  Host-side, single-threaded use.
 */
int fp8a_kernel_timing(int enable);
int fp8a_kernel_time(double *out, int reset);

/*
 * Runtime options (A/B measurements, tests, diagnostics):
 * "tbx_rw" (default 2; FP8A_TBX_RW) -- output rows per thread of the table-form depthwise kernel;
 * "tbs" (default 2; FP8A_TBS) -- the table-form depthwise kernel: 2 = window staged by LDS-DMA,
 * 1 = register-staged, both with the word pre-pass fused; 0 = the word-image gather (same bits); "dw3" (default 2; FP8A_DW3) -- the exact depthwise 3x3: 2 = window staged by LDS-DMA,
 * 4 outputs per thread; 1 = register-staged window; 0 = the general grouped kernel (same bits);
 * "dw_target" / "dw_lds" -- outputs / LDS bytes per workgroup of those staged kernels;
 * "dn_direct" (default 1; FP8A_DN_DIRECT) -- exact convolutions with Cin kh kw <= 32 and Cout <= 64
 * (the stem) as direct fp32 FMAs instead of the bf16 matrix-core GEMM;
 * "v5ds" (default 1; FP8A_V5DS) -- the v5 (E5M2, adder wrap) depthwise 3x3 on the staged kernel
 * with both word pre-passes fused (0: the pre-passes + the word-form kernel; same bits);
 * "xm_ncg" (default 0 = by N; FP8A_XM_NCG) -- gemm_f8mx_kernel's tile width forced to 16 x 1 / 2
 * / 4 columns; "af32_maxct" (default 1, times sh x sw for a strided conv; FP8A_AF32_MAXCT) -- the most column tiles for which a 1x1
 * conv / matrix A is decoded inside gemm_f8mx_kernel instead of by its pre-pass (0 = never);
 * "tt16_mink" (default 64; FP8A_TT16_MINK) -- the smallest K of an E3M4 launch (unsigned error
 * table) on the packed-f16 tile-table kernel (shorter K: the f32 form); "tt_band" (default 1;
 * FP8A_TT_BAND) -- gemm_tt_kernel's band / zero wave-tile forms (0 = the general form everywhere).
 * All of these change the schedule only: the outputs are bit-identical.  Returns the previous value, or FP8A_EINVAL
 * for an unknown name.  Not synchronised with launches in flight on other threads.
 */
int fp8a_set_option(const char *name, int value);

/*
 * The exact (non-approx) product on the matrix core -- the reference's `x @ y` of FP8-quantized
 * operands (approx_calculation.py:797, 811: QuantizationHijacker with approx_flag off, BASELINE
 * config 1; the im2col form for convs).  Operands are fp32 values.  fmt FP8A_DENSE_BF16 (what the
 * Python operators use by default): truncated to bf16 -- exact for every value with <= 8
 * significant bits, i.e. every FP8 / E3M4 / E2M5 grid value at any exponent -- and multiplied by
 * v_mfma_f32_16x16x32_bf16.  fmt FP8A_DENSE_E4M3 / _E5M2 (opt-in): per (row, 32-k block)
 * converted to OCP e4m3 / e5m2 with a power-of-two block scale and multiplied by the block-scaled
 * MFMA.  Both accumulate in fp32.  Values that are not exact in the operand format
 * (off-grid, too far below the block's largest, inf / NaN) send their 64-row / 64-column output
 * units to an fp32 FMA recompute, so ANY finite or non-finite input gives the fp32 product up to
 * summation order.  fp8a_dense_matmul: A element (m, k) at A[m * sam + k * sak], B element (k, n)
 * at B[k * sbk + n * sbn], C row-major with ldc.  fp8a_dense_conv2d: NCHW x, w [Cout][Cin][kh][kw],
 * NCHW y, groups = 1.  Workspace: the *_workspace_size bytes.
 */
#define FP8A_DENSE_E4M3 0
#define FP8A_DENSE_E5M2 1
#define FP8A_DENSE_BF16 2  /* bf16 operands (any value with <= 8 significant bits, every exponent) */
size_t fp8a_dense_matmul_workspace_size(int64_t M, int64_t N, int64_t K);
int fp8a_dense_matmul(const float *A, int64_t sam, int64_t sak, const float *B, int64_t sbk, int64_t sbn, float *C,
                      int64_t ldc, int64_t M, int64_t N, int64_t K, int fmt, void *workspace, size_t workspace_bytes,
                      fp8a_stream_t stream);
size_t fp8a_dense_conv2d_workspace_size(int64_t Bn, int64_t Cin, int64_t H, int64_t W, int64_t Cout, int kh, int kw,
                                        int sh, int sw, int ph, int pw, int dh, int dw);
int fp8a_dense_conv2d(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H, int64_t W,
                      int64_t Cout, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw, int fmt,
                      void *workspace, size_t workspace_bytes, fp8a_stream_t stream);
/* The exact grouped / depthwise convolution (QCustomConv2dTorch's per-group im2col + x @ w^T,
 * approx_calculation.py:686-711; the exact branch's x @ y[:, i] for groups > 1, :797): NCHW x,
 * w [Cout][Cin / groups][kh][kw], NCHW y, fp32 FMAs in the im2col k order (channel, ky, kx), the
 * padding as zeros.  Any fp32 input; no workspace.  Counted as a dense launch (fp8a_path_stats).
 * Depthwise 3x3 with equal strides 1 / 2 runs an LDS-staged kernel (option "dw3", the same bits). */
int fp8a_grouped_conv2d(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H, int64_t W,
                        int64_t Cout, int groups, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw,
                        fp8a_stream_t stream);
/* A config-1 layer (approx_flag off: BNFusedHijacker's forward around the exact product,
 * quantized_folded_bn.py:30-83 / hijacker.py:77-115) in one pass over its output:
 *   y = fq_out(clamp(bn(fq_res(conv(fq_in(x), w)))))
 * fq_in = the input's activation quantizer (quantize_input), fq_res = the res quantizer
 * (original_quantize_res), bn = eval batch norm as [Cout][2] {scale, shift} floats, clamp =
 * [act_lo, act_hi] when act, fq_out = the output's activation quantizer, and w read through the
 * weight quantizer fq_w (get_params' quantize_weights, hijacker.py:113-120); every member optional
 * (maxval / bn NULL).  FP8 quantizers (quantize_to_fp8_ste_MM): per tensor, fq_w also per output
 * channel (w_per_channel: w_maxval [Cout], biases [Cout]); each writes its bias (custom_bias) to
 * *_bias_out / *_ibias_out from inside the layer's first kernel.  groups = 1: the dense product
 * (fmt as fp8a_dense_conv2d, its workspace); groups > 1: fp8a_grouped_conv2d's kernel (no
 * workspace). */
int fp8a_dense_conv2d_fused(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H, int64_t W,
                            int64_t Cout, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw, int groups,
                            int fmt, const float *w_maxval, int w_per_channel, int w_nbits, int w_mbits,
                            int w_sign_bits, float *w_bias_out, int32_t *w_ibias_out, const float *in_maxval,
                            int in_nbits, int in_mbits, int in_sign_bits, float *in_bias_out, int32_t *in_ibias_out,
                            const float *res_maxval, int res_nbits, int res_mbits, int res_sign_bits,
                            float *res_bias_out, int32_t *res_ibias_out, const float *bn, int act, float act_lo,
                            float act_hi, const float *out_maxval, int out_nbits, int out_mbits, int out_sign_bits,
                            float *out_bias_out, int32_t *out_ibias_out, void *workspace, size_t workspace_bytes,
                            fp8a_stream_t stream);
/* Dense-path counters since load / the last reset (out[2]): [0] launches with units recomputed in
 * fp32, [1] 64 x 64 units recomputed.  Synchronises the device. */
int fp8a_dense_stats(uint64_t *out, int reset);

/* Diagnostic: the in-kernel clock of gemm_f8mx_kernel, counted only by a library built with
 * -DFP8A_CLOCK_STAMP=1 (tools/clock_probe.py; zeros otherwise), out[3]: sum over workgroups of
 * the s_memtime delta, of the s_memrealtime (100 MHz) delta, and the workgroup count.
 * Synchronises the device. */
int fp8a_clock_stats(uint64_t *out, int reset);

/*
 * Element decomposition DEC of float_to_fpany_absint_torch (approx_matmul_whole_v9.py:233-291)
 * over a rows x cols matrix with row stride ld.  bias: device int32, bias_stride 0 = one bias
 * for all elements, 1 = one bias per ROW (per-channel weights).  flags: FP8A_TB selects the
 * tensor-bias variant of param_prepare (v9:189-229); FP8A_GCLIP selects clip_OF.
 * Writes expo/mant (int32, dense rows x cols).
 */
int fp8a_decompose(const float *x, int64_t rows, int64_t cols, int64_t ld, int E, int M,
                   const int32_t *bias, int64_t bias_stride, uint32_t flags,
                   int32_t *expo, int32_t *mant, fp8a_stream_t stream);

/* Q_R = quant_to_fp_any_vectorize_torch (v9:333-362) elementwise over n floats. */
int fp8a_quant(const float *x, int64_t n, int E, int M, const int32_t *bias, uint32_t flags,
               float *out, fp8a_stream_t stream);

/*
 * Replaces custom_matmul_vectorize (approx_matmul_whole_v9.py:10-169) as driven by
 * approx_multiply's per-column loop (approx_calculation.py:749-814 / 921-999):
 *   C[m, n] = sum_k term(A[m, k], B(k, n)),   B(k, n) = B[k * sbk + n * sbn]
 * with bA (device int32 [1]), bB (device int32, bB_stride 0 = shared, 1 = per column), bR
 * (device int32 [1]).  table: HOST int32 [2^M][2^M] error table (get_error_table_NN,
 * v9:555-592) or NULL for all-zero; it is packed into the launch arguments, so the call stays
 * asynchronous.  C is row-major with leading dimension ldc.  workspace: device scratch of at
 * least fp8a_matmul_workspace_size() bytes (holds the off-grid flag that gates the exact
 * re-computation when an operand is not exactly representable in its FP8 code -- with this
 * minimal workspace any fallback recomputes the whole product); a workspace of
 * fp8a_matmul_workspace_size_mnk(M, N, K) bytes also holds the per-64x64-unit fallback marks
 * (only the affected output units are recomputed) and split-K partial sums, which the launch
 * then uses when the shape fills the GPU in a fractional number of waves (the partials are
 * summed in a fixed order: results stay deterministic).
 */
size_t fp8a_matmul_workspace_size(void);
size_t fp8a_matmul_workspace_size_mnk(int64_t M, int64_t N, int64_t K);
int fp8a_matmul(const float *A, int64_t lda, const float *B, int64_t sbk, int64_t sbn,
                float *C, int64_t ldc, int64_t M, int64_t N, int64_t K, int E, int Mw,
                const int32_t *bA, const int32_t *bB, int64_t bB_stride, const int32_t *bR,
                const int32_t *table, uint32_t flags, void *workspace, size_t workspace_bytes,
                fp8a_stream_t stream);

/*
 * Per-product terms (debug / parity): T[m, k, n] = the value the reference sums at v9:113.
 * Same arguments as fp8a_matmul; T is dense [M][K][N].
 */
int fp8a_terms(const float *A, int64_t lda, const float *B, int64_t sbk, int64_t sbn, float *T,
               int64_t M, int64_t N, int64_t K, int E, int Mw, const int32_t *bA,
               const int32_t *bB, int64_t bB_stride, const int32_t *bR, const int32_t *table,
               uint32_t flags, fp8a_stream_t stream);

/*
 * Replaces QCustomBNConv2dTorch.run_forward (approx_calculation.py:822-917) minus the conv
 * bias: x NCHW [Bn, Cin, H, W], w [Cout, Cin/groups, kh, kw], y NCHW [Bn, Cout, Ho, Wo].
 * bW: device int32 per output channel (weight_quantizer.custom_bias).  Groups whose output
 * block has a single channel (depthwise) take the tensor-bias semantics (FP8A_TB) exactly as
 * the reference does (approx_calculation.py:800-809), other groups the int-bias semantics.
 * workspace: device scratch of fp8a_conv2d_workspace_size() bytes (the off-grid flag word
 * and split-K partial sums; no im2col image: the GEMM gathers its operand rows from x).  A
 * smaller workspace that still holds the flag word runs without split-K.  Its first word receives
 * the launch's final flag word; the flags and unit marks themselves live in the library's
 * per-stream flag arena (no fill per launch; the first call on a stream allocates it) -- except
 * while a HIP graph is being captured on the stream: a captured launch keeps them in the head of
 * its workspace (fp8a_*_workspace_size's layout reserves it), zeroed by a fill kernel at the start of
 * the launch (no graph memset node: DESIGN.md §3r), so every replay
 * starts from zero flags and graphs never reference the arena (capture-safe).
 */
size_t fp8a_conv2d_workspace_size(int64_t Bn, int64_t Cin, int64_t H, int64_t W, int64_t Cout,
                                  int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw,
                                  int groups);
int fp8a_conv2d(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H,
                int64_t W, int64_t Cout, int kh, int kw, int sh, int sw, int ph, int pw, int dh,
                int dw, int groups, int E, int Mw, const int32_t *bA, const int32_t *bW,
                const int32_t *bR, const int32_t *table, uint32_t flags, void *workspace,
                size_t workspace_bytes, fp8a_stream_t stream);

/*
 * fp8a_conv2d with the layer's eval-mode BatchNorm and activation fused into the epilogue
 * (BNFusedHijacker.forward: F.batch_norm after run_forward, then the activation,
 * quantization/quantized_folded_bn.py:30-83): y = acc * scale + shift per output channel, with
 * scale = gamma / sqrt(running_var + eps) and shift = beta - running_mean * scale (the eval-mode
 * transform ATen applies), then clamped to [act_lo, act_hi] when act != 0 (ReLU: [0, inf],
 * ReLU6: [0, 6], Hardtanh: [min_val, max_val]).  bn: device float [Cout][2] = {scale, shift},
 * 8-byte aligned, or NULL (plain fp8a_conv2d).
 */
int fp8a_conv2d_bn_act(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin,
                       int64_t H, int64_t W, int64_t Cout, int kh, int kw, int sh, int sw, int ph,
                       int pw, int dh, int dw, int groups, int E, int Mw, const int32_t *bA,
                       const int32_t *bW, const int32_t *bR, const int32_t *table, uint32_t flags,
                       const float *bn, int act, float act_lo, float act_hi, void *workspace,
                       size_t workspace_bytes, fp8a_stream_t stream);

/*
 * fp8a_conv2d_bn_act with the layer's input activation quantizer fused in (the hijacker's
 * `x = activation_quantizer(x)` before run_forward, hijacker.py:81-83, in the fixed-range eval
 * state): x is the UNQUANTIZED input; the op applies quantize_to_fp8_ste_MM
 * (fp8_quantizer.py:97-173) with the per-tensor in_maxval (device float [1]) and format, writes
 * the quantizer's bias to in_bias_out (float [1]) / in_ibias_out (int32 [1], what it returns as
 * custom_bias) and uses it as bA.  Same result as fp8a_fp8_quantize followed by
 * fp8a_conv2d_bn_act; where the E4M3 matrix-core or tensor-bias table kernels run, the
 * quantization happens inside their operand pre-decode (no quantized copy of x is written).
 * workspace: fp8a_conv2d_qin_workspace_size() bytes.
 */
size_t fp8a_conv2d_qin_workspace_size(int64_t Bn, int64_t Cin, int64_t H, int64_t W, int64_t Cout,
                                      int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw,
                                      int groups);
int fp8a_conv2d_qin(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H,
                    int64_t W, int64_t Cout, int kh, int kw, int sh, int sw, int ph, int pw, int dh,
                    int dw, int groups, int E, int Mw, const int32_t *bW, const int32_t *bR,
                    const int32_t *table, uint32_t flags, const float *bn, int act, float act_lo,
                    float act_hi, const float *in_maxval, int in_nbits, int in_mbits,
                    int in_sign_bits, float *in_bias_out, int32_t *in_ibias_out, void *workspace,
                    size_t workspace_bytes, fp8a_stream_t stream);

/*
 * A residual block's last convolution with the block's tail fused into its store
 * (resnet_quantized_approx.py:11-41 QuantizedBlock: out = relu(features(x) + residual), then the
 * block's activation quantizer; mobilenet_v2_quantized_approx.py:11-23: quantize(x + conv(x))):
 *   y = fq_out(clamp(bn_act(conv(fq_in(x))) + res, post_lo, post_hi))
 * in_maxval NULL: x is already quantized and bA is used (else as fp8a_conv2d_qin).  res: NULL or
 * a 16-byte aligned tensor of y's shape (not y itself).  post_act 0: no clamp, 1: the clamp
 * (anything else: FP8A_EINVAL).  out_maxval NULL:
 * no output quantizer; else its bias is written to out_bias_out / out_ibias_out.  Not for
 * single-output-channel groups (EINVAL).  workspace: fp8a_conv2d_block_workspace_size() bytes.
 */
size_t fp8a_conv2d_block_workspace_size(int64_t Bn, int64_t Cin, int64_t H, int64_t W, int64_t Cout,
                                        int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw,
                                        int groups);
int fp8a_conv2d_block(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H,
                      int64_t W, int64_t Cout, int kh, int kw, int sh, int sw, int ph, int pw, int dh,
                      int dw, int groups, int E, int Mw, const int32_t *bA, const int32_t *bW,
                      const int32_t *bR, const int32_t *table, uint32_t flags, const float *bn,
                      int act, float act_lo, float act_hi, const float *in_maxval, int in_nbits,
                      int in_mbits, int in_sign_bits, float *in_bias_out, int32_t *in_ibias_out,
                      const float *res, int post_act, float post_lo, float post_hi,
                      const float *out_maxval, int out_nbits, int out_mbits, int out_sign_bits,
                      float *out_bias_out, int32_t *out_ibias_out, void *workspace,
                      size_t workspace_bytes, fp8a_stream_t stream);

/*
 * Word-image hand-off between two convolutions (round 4; no reference counterpart: it removes the
 * A operand pre-pass xm_decode_a that the matrix-core path runs on every convolution's input).
 * A word image is a convolution's input pre-decoded for the matrix-core kernel -- one 32-bit word
 * per element in a zero-bordered [Bn][C][H + 2 ph][W'] layout -- behind a 256-byte header whose
 * first word flags it invalid.  fp8a_word_image_bytes gives its size (0 for bad arguments);
 * fp8a_word_image_init fills a 256-byte aligned buffer once (header valid, every word that of a
 * zero: the border keeps it).
 */
size_t fp8a_word_image_bytes(int64_t Bn, int64_t C, int64_t H, int64_t W, int ph, int pw);
int fp8a_word_image_init(void *image, int64_t Bn, int64_t C, int64_t H, int64_t W, int ph, int pw,
                         fp8a_stream_t stream);

/*
 * fp8a_conv2d_block with the hand-off (the reference's QuantizedBlock / Sequential chain of
 * QCustomBNConv2dTorch layers, resnet_quantized_approx.py:11-41, each quantizing its own input,
 * hijacker.py:81-83):
 *   in_image: NULL, or THIS convolution's input x as the word image a previous fp8a_conv2d_chain
 *             call emitted (same Bn, Cin, H, W, ph, pw; needs in_maxval: the words hold
 *             fq_in(x)).  Where the matrix-core path runs, its words replace the A pre-pass; an
 *             image flagged invalid (an element outside the path's window) is re-decoded from x,
 *             which must be the fp32 tensor the emitting call wrote -- that re-decode rewrites the
             image's words in place (hence non-const).  Elsewhere it is ignored.
 *   out_image: NULL, or the NEXT convolution's input image to emit while y is stored: the words
 *             of next_fq(y) for a next convolution with padding next_ph / next_pw, input quantizer
 *             next_maxval (per tensor) / next_nbits / next_mbits / next_sign_bits, result bias
 *             next_bR and mantissa width next_Mw (3: E4M3, 2: E5M2); next_form = the next
 *             convolution's fp8a_conv2d_wants_image - 1 (0: matrix-core words in an image of
 *             next_ph / next_pw; 1: table-form words, image of ph = pw = 0; 2: the v5 matrix-core
 *             form's words, emitted by a v5 depthwise 3x3 producer on its staged kernel).  y is
 *             written as well; form 0 is also emitted by a tensor-bias depthwise 3x3 producer on
 *             its staged table-form kernel (round 6).  Where this call cannot emit (other grouped
 *             producers, Cout == 1, a tile-table or v5 matrix-core producer, whose store does not
 *             emit, a depthwise launch on another kernel) the image is flagged invalid.
 * Results are bit-identical to the unchained calls.  workspace: fp8a_conv2d_block_workspace_size().
 */
/* The word image a convolution of this shape / format would read as in_image: 1 = the matrix-core
 * path's (ungrouped, Cout > 1, E4M3 / E5M2 with s2n + qbma and a {0,1} or zero table, not a 1x1
 * unpadded convolution staged from fp32; images of its padding), 2 = the tensor-bias table form's
 * (single-output-channel groups, 3-wide undilated rows, stride 1 / 2; images with ph = pw = 0),
 * 3 = the v5 matrix-core form's (unpadded convolutions), 0 = none: emitting an image for it would
 * be wasted. */
int fp8a_conv2d_wants_image(int64_t Cout, int kh, int kw, int ph, int pw, int groups, int E, int Mw,
                            const int32_t *table, uint32_t flags, int sh, int sw, int dh, int dw);
int fp8a_conv2d_chain(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H,
                      int64_t W, int64_t Cout, int kh, int kw, int sh, int sw, int ph, int pw, int dh,
                      int dw, int groups, int E, int Mw, const int32_t *bA, const int32_t *bW,
                      const int32_t *bR, const int32_t *table, uint32_t flags, const float *bn,
                      int act, float act_lo, float act_hi, const float *in_maxval, int in_nbits,
                      int in_mbits, int in_sign_bits, float *in_bias_out, int32_t *in_ibias_out,
                      const float *res, int post_act, float post_lo, float post_hi,
                      const float *out_maxval, int out_nbits, int out_mbits, int out_sign_bits,
                      float *out_bias_out, int32_t *out_ibias_out, void *in_image,
                      void *out_image, int next_ph, int next_pw, const float *next_maxval,
                      int next_nbits, int next_mbits, int next_sign_bits, const int32_t *next_bR,
                      int next_Mw, int next_form, void *workspace, size_t workspace_bytes,
                      fp8a_stream_t stream);

/*
 * A linear layer with its neighbours' elementwise work fused (QCustomLinearTorch.run_forward,
 * approx_calculation.py:1007-1023, plus the callers' tails in vit_quantized_approx.py:117-156):
 *   C = fq_out(clamp(bn_act(fq_in(A) @ B) + res, post_lo, post_hi))
 * Operands as fp8a_matmul.  bn: NULL or [N][2] {scale, shift} per output column (the linear's bias
 * is {1, bias}: x * 1 + bias is the reference's `out += bias`), act / act_lo / act_hi a clamp.
 * in_maxval NULL: A is already quantized and bA is used; else A (dense: lda == K) is quantized
 * by that per-tensor FP8 quantizer inside the operand pre-decode where the E4M3 matrix-core
 * path runs (else by one pass into the workspace) and its bias is written to in_bias_out /
 * in_ibias_out.  res: NULL or a 16-byte aligned [M][ldc] tensor (not C).  post / out_* as
 * fp8a_conv2d_block, plus post_act 2: GELU (nn.GELU(), erf form, as ATen evaluates it in fp32)
 * in place of the clamp -- vit_quantized_approx.py:117-135's dense, GELU, quantize in one launch.
 * int-bias v9 path only (no TB / V5 flags).
 * workspace: fp8a_matmul_block_workspace_size() bytes.
 */
size_t fp8a_matmul_block_workspace_size(int64_t M, int64_t N, int64_t K);
int fp8a_matmul_block(const float *A, int64_t lda, const float *B, int64_t sbk, int64_t sbn, float *C,
                      int64_t ldc, int64_t M, int64_t N, int64_t K, int E, int Mw, const int32_t *bA,
                      const int32_t *bB, int64_t bB_stride, const int32_t *bR, const int32_t *table,
                      uint32_t flags, const float *bn, int act, float act_lo, float act_hi,
                      const float *in_maxval, int in_nbits, int in_mbits, int in_sign_bits,
                      float *in_bias_out, int32_t *in_ibias_out, const float *res, int post_act,
                      float post_lo, float post_hi, const float *out_maxval, int out_nbits,
                      int out_mbits, int out_sign_bits, float *out_bias_out, int32_t *out_ibias_out,
                      void *workspace, size_t workspace_bytes, fp8a_stream_t stream);

/*
 * nn.MaxPool2d (dilation 1, floor mode, padding <= half the window) on NCHW fp32 y[Bn][C][Ho][Wo]:
 * the ResNet stem pooling on the benchmarked step (not an approx op).
 */
int fp8a_max_pool2d(const float *x, float *y, int64_t Bn, int64_t C, int64_t H, int64_t W, int kh,
                    int kw, int sh, int sw, int ph, int pw, fp8a_stream_t stream);

/*
 * nn.AvgPool2d (no padding, floor mode, no divisor override) whose output is one value per plane
 * -- the window is each plane's top-left kh x kw (kh <= H < kh + sh, likewise W): the
 * MobileNetV2 head's AvgPool2d(input_size // 32) on the benchmarked step (not an approx op).
 * y[Bn][C][1][1] = the window summed in row-major order in fp32, divided by kh kw (ATen's
 * avg_pool2d: the same bits).  FP8A_EINVAL for any other geometry or planes over 4096 values.
 */
int fp8a_avg_pool2d_plane(const float *x, float *y, int64_t Bn, int64_t C, int64_t H, int64_t W,
                          int kh, int kw, int sh, int sw, fp8a_stream_t stream);

/*
 * quantize_after_mult_and_add (qamaa) path of approx_multiply (approx_calculation.py:787-795):
 *   C = fq(sum_k fq(A[m,k] * B(k,n))),  fq = quantize_to_fp8_ste_MM with the res quantizer's
 *   n_bits / mantissa bits / sign bits and per-tensor maxval (device float [1]).
 * C is dense [M][N].  Exact for any fp32 inputs (no operand decode).
 */
int fp8a_matmul_qamaa(const float *A, int64_t lda, const float *B, int64_t sbk, int64_t sbn,
                      float *C, int64_t M, int64_t N, int64_t K, const float *maxval, int n_bits,
                      int Mbits, int sign_bits, fp8a_stream_t stream);
/* Convolution form (groups with > 1 output channel; single-output-channel groups take the
 * reference's exact product and are not launched here). */
int fp8a_conv2d_qamaa(const float *x, const float *w, float *y, int64_t Bn, int64_t Cin, int64_t H,
                      int64_t W, int64_t Cout, int kh, int kw, int sh, int sw, int ph, int pw,
                      int dh, int dw, int groups, const float *maxval, int n_bits, int Mbits,
                      int sign_bits, fp8a_stream_t stream);

/* The reference's im2col (approx_calculation.py:724-747): out [Bn*Ho*Wo, Cin*kh*kw]. */
int fp8a_im2col(const float *x, float *out, int64_t Bn, int64_t Cin, int64_t H, int64_t W,
                int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw,
                fp8a_stream_t stream);

/*
 * FP8 fake quantizer forward value, quantize_to_fp8_ste_MM (fp8_quantizer.py:97-173),
 * E = n_bits - sign_bits - Mbits, clamp range [-maxval, maxval] (sign_bits 1) or [0, maxval]:
 * x viewed as [rows, inner]; maxval device float [rows] if per_row else [1].  Writes out (same shape) and, if bias_out != NULL, the float bias
 * round(2^E - log2(maxval) + log2(2 - 2^-M) - 1) per row (or [1]) and, if ibias_out != NULL,
 * the same bias as int32 (what approx_multiply feeds the matmul, approx_calculation.py:768).
 */
int fp8a_fp8_quantize(const float *x, int64_t rows, int64_t inner, const float *maxval,
                      int per_row, int n_bits, int Mbits, int sign_bits, float *out,
                      float *bias_out, int32_t *ibias_out, fp8a_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* FP8APPROX_H */
