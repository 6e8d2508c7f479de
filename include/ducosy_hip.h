/*
 * ducosy_hip.h — C-ABI of the MI355X (gfx950) kernel library behind the DuCoSy-GAN
 * CycleGAN training hot path.
 *
 * The reference has no FFI: its de-facto operator boundary is the Python nn.Module /
 * loss-module API of modules/model.py and modules/trainer.py, which reach ATen/cuDNN
 * kernels through torch.nn.  Every entry point below replaces one such group of ATen
 * calls (cited per function, paths relative to the reference repo).  The host side
 * (ducosy-gan_amd/modules/hip/ Python modules) binds them with ctypes.
 *
 * Conventions
 *   - Plain device pointers + int sizes; no torch types.  Activations are NHWC fp32
 *     (channels innermost); single-channel planes are NCHW == NHWC.
 *   - The caller owns every buffer (including workspaces, sized by *_workspace_size).
 *     The library never allocates or frees device memory and never synchronises.
 *   - Every call is enqueued on `stream` (a hipStream_t passed as void*).
 *   - Every call returns 0 on success, a DCS_E_* code on an invalid argument, or the
 *     hipError_t of a failed launch; dcs_last_error() returns a thread-local message.
 */
#ifndef DUCOSY_HIP_H
#define DUCOSY_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DCS_OK 0
#define DCS_E_INVALID 1001
#define DCS_E_WORKSPACE 1002

#define DCS_PAD_ZERO 0
#define DCS_PAD_REFLECT 1

/* per-channel prologue transform applied to gathered source values:
 * v -> act(v * scale[n,c] + shift[n,c]); padding stays zero (or mirrors transformed values) */
#define DCS_ACT_NONE 0     /* no transform at all */
#define DCS_ACT_AFFINE 1   /* affine only (InstanceNorm apply) */
#define DCS_ACT_RELU 2     /* affine + ReLU                    */
#define DCS_ACT_LRELU 3    /* affine + LeakyReLU(0.2)          */
#define DCS_ACT_TANH 4     /* epilogue only                    */

/*
 * Geometry of one implicit-GEMM convolution pass.
 *   source  : the tensor gathered into the GEMM reduction (forward: x, dgrad: dy)
 *   output  : NHWC [N, Ho, Wo, Co]
 * Regular rows (parity = 0): output pixel (oy, ox) reads virtual source coordinate
 *   (oy*stride + ty - pt, ox*stride + tx - pl) for tap (ty, tx); the virtual source is
 *   the source upsampled (nearest) by `up`, padded by pad_mode.
 * Parity rows (parity = 1): stride-2 transposed convolution (dgrad of a stride-2
 *   forward conv with kernel KH x KW and padding pt/pl): output pixel (2qy+ry, 2qx+rx)
 *   reads dy at (qy + (ry+pt-ty)/2, qx + (rx+pl-tx)/2) for the taps of its parity class.
 */
typedef struct dcs_conv_desc {
    int32_t N;
    int32_t Hs, Ws, Cs;             /* source dims (Cs = reduction channels per tap)      */
    int64_t s_n, s_c, s_h, s_w;     /* source element strides                             */
    int32_t csplit;                 /* channels >= csplit come from src2 (concat fusion)  */
    int32_t cw;                     /* weight input channels if < Cs (zero-padded source  */
                                    /* channels, e.g. the 3-channel stem packed to 4); 0 = Cs */
    int64_t s2_n, s2_c, s2_h, s2_w; /* src2 strides (channel index relative to csplit)   */
    int32_t up;                     /* nearest-upsample factor of the source (1 or 2)     */
    int32_t pad_mode;               /* DCS_PAD_ZERO / DCS_PAD_REFLECT                     */
    int32_t KH, KW, pt, pl;         /* kernel, top/left padding                           */
    int32_t stride;                 /* forward stride (1 or 2)                            */
    int32_t parity;                 /* 0 regular rows, 1 stride-2 transposed parity rows  */
    int32_t Ho, Wo, Co;             /* output dims                                        */
    int32_t ldb;                    /* packed weights: Kpad (rows pass) / ncols (narrow)  */
    int32_t pro_act;                /* DCS_ACT_* prologue on the source                   */
    int32_t epi_act;                /* DCS_ACT_NONE / DCS_ACT_TANH / DCS_ACT_LRELU        */
    int32_t mma;                    /* MFMA operands: DCS_MMA_F32 (exact; 0 = zeroed desc) */
                                    /* or DCS_MMA_BF16 / _BF16X3 / _BF16X6 (f32 accum.)   */
    int32_t korder;                 /* GEMM K order of the rows pass (and of its packed    */
                                    /* weights): DCS_KORDER_TAP (tap-major) or            */
                                    /* DCS_KORDER_SLICE (16-channel slices, taps inside)  */
    int32_t rng_a_n, rng_b_n;       /* DCS_MMA_F16X3: counts of the partial maxima below   */
    const float* rng_a;             /* F16X3: partial maxima of |gathered operand| (rows:  */
                                    /* the source after its prologue; wgrad: dy), their   */
                                    /* max an upper bound of every value (dcs_range_parts) */
    const float* rng_b;             /* F16X3: the same for the other operand (rows: the   */
                                    /* packed weights, dcs_pack_weights_r; wgrad: source) */
    const void* b_h3;               /* F16X3 / F16 rows pass, optional: the packed weights */
                                    /* pre-split by dcs_pack_split_h3 (B staged without a */
                                    /* split); NULL: split at staging                     */
} dcs_conv_desc;

/* K order of the rows pass.  TAP: k = tap * Cs + c.  SLICE: k = (c / 16) * taps * 16 + tap * 16 +
 * c % 16 — every tap of a 16-channel slice before the next slice, so the gathered source rows
 * of a slice are re-read from L2 / L1 by the next taps instead of after a whole tap sweep
 * (regular stride-1 rows, Cs % 16 == 0; pack the weights with DCS_PACK_KSLICE). */
#define DCS_KORDER_TAP 0
#define DCS_KORDER_SLICE 1
#define DCS_PACK_KSLICE 8

/* MFMA operand modes of the MFMA convolution passes (dcs_conv_desc.mma).  F32 is exact fp32
 * (the reference's precision).  BF16 rounds both GEMM operands to bf16 (BASELINE config 5's
 * half-precision path).  BF16X3 splits each operand into hi + lo bf16 and sums three
 * products (~2^-16 relative error per product).  Shapes without a bf16 variant run F32. */
#define DCS_MMA_F32 0
#define DCS_MMA_BF16 1
#define DCS_MMA_BF16X3 3
/* BF16X6: three-way split (hi + mid + lo bf16), six products, ~2^-24 relative error per
 * product (fp32-class); 128-column tiles only, other shapes run F32. */
#define DCS_MMA_BF16X6 6
/* F16X3: each fp32 operand, scaled by a power of two 2^s (max|operand| * 2^s < 2^15, from the
 * descriptor's rng_a / rng_b partial maxima), is split into hi + lo fp16 (22 significant bits:
 * |v - hi - lo| <= 2^-22 |v|); three products hi*hi + hi*lo + lo*hi on v_mfma_f32_32x32x16_f16,
 * fp32 two-level accumulation, the result scaled back by 2^-(s_a + s_b) (exact).  Measured
 * error against float64 at or below the exact-f32 path's on every layer geometry
 * (tests/test_gpu_mma.py): fp32-class at half the MFMAs of BF16X6.  Shapes without an F16X3
 * variant run BF16X6. */
#define DCS_MMA_F16X3 7
/* F16: BASELINE config 5's fp16 MFMA path.  Each fp32 operand, scaled by the same power of two as
 * F16X3 (from rng_a / rng_b), is rounded to fp16 (11 significant bits, no overflow or underflow
 * from the scale); one product per fragment pair on v_mfma_f32_32x32x16_f16, fp32 accumulation and
 * storage, the result scaled back exactly.  Shapes without an F16 variant run BF16X6. */
#define DCS_MMA_F16 8
/* partial maxima the F16X3 kernels reduce (dcs_range_parts writes this many).  The producers of
 * conv operands (dcs_in_apply, dcs_in_act_backward, dcs_cbam_forward, dcs_cbam_backward,
 * dcs_act_backward, dcs_pack_nhwc4) take an optional `rng` (DCS_RANGE_PARTS floats, or NULL):
 * they zero it and fold the max |value| they write into it, so an F16X3 pass over their output
 * needs no separate dcs_range_parts read. */
#define DCS_RANGE_PARTS 512

const char* dcs_last_error(void);
int dcs_version(void);


/* ---- convolution family (modules/model.py:61-63,74-79,94-112,122-129 → aten conv) ---- */

/* Pack OIHW weights into the GEMM B operand, logically [Kpad][ncols] (zero padded), stored
 * N-major ([ncols][Kpad]; nmajor=1, for dcs_conv_rows, ldb = Kpad) or K-major ([Kpad][ncols];
 * nmajor=0, for the narrow kernels, ldb = ncols).
 * kind 0 forward   : B[(ty*KW+tx)*Cin + ci][co] = W[co][ci][ty][tx]
 * kind 1 dgrad-flip: B[(ty*KW+tx)*Cout + co][ci] = W[co][ci][KH-1-ty][KW-1-tx]  (stride-1 dgrad)
 * kind 2 dgrad     : B[(ty*KW+tx)*Cout + co][ci] = W[co][ci][ty][tx]              (stride-2 dgrad)
 * kind 3 / 4      : sub-pixel forward / data gradient of nearest-x2 upsample + 3x3 conv
 * kind 5 fwd-pad  : B[(ty*KW+tx)*ci_count + ci][co] = ci < Cin ? W[co][ci][ty][tx] : 0
 *                   (forward over a source whose channels are zero-padded to ci_count)
 * kind | DCS_PACK_KSLICE (kinds 0 and 1): the same B with its K rows in DCS_KORDER_SLICE order
 * ci_count limits the packed input channels (dgrad of a concat input needs only the first). */
int dcs_pack_weights(const float* w, int Cout, int Cin, int KH, int KW, int kind, int ci_count,
                     int Kpad, int ncols, int nmajor, float* out, void* stream);
/* The same, and DCS_RANGE_PARTS partial maxima of |packed value| into rng (the rng_b of an
 * F16X3 rows pass over these weights). */
int dcs_pack_weights_r(const float* w, int Cout, int Cin, int KH, int KW, int kind, int ci_count,
                       int Kpad, int ncols, int nmajor, float* out, float* rng, void* stream);

/* Fused G-step loss planes (the north star's fused cycle / identity / SSIM / gradient /
 * contrast-loss kernel; replaces the per-term calls of modules/trainer.py:469-512).  One job per
 * (pred, target) plane set of n_img single-channel H x W planes; flags select its terms:
 *   DCS_GL_L1 nn.L1Loss, DCS_GL_GRAD GradientLoss (trainer.py:22-40), DCS_GL_SSIM
 *   pytorch_msssim.SSIM (11-tap sigma 1.5 valid gaussian, size_average), DCS_GL_CA
 *   ContrastAttentionLoss with a 7x7 box (trainer.py:43-86; needs source), DCS_GL_MSEC
 *   nn.MSELoss against the constant t_const (target unused).
 * grad (optional) receives c_l1 d(L1)/dpred + c_grad d(Grad)/dpred + c_ssim d(SSIM)/dpred +
 * c_ca d(CA)/dpred + c_mse d(MSE)/dpred + c_add0 add0 + c_add1 add1 in one write per pixel
 * (add0 / add1: optional planes of the same shape, e.g. the batch-coupled terms' gradients).
 * Term values (means) val[5 j + q], q = 0 L1, 1 gradient-loss x part, 2 y part, 3 SSIM, 4 CA or
 * MSE, are composed into out[o] = bias[o] + sum_k coef[o * 5 njobs + k] val[k]
 *                                 + sum_x coefx[o * 4 + x] extra[x][0]  (o < nout <= 12)
 * (extra: up to 4 device scalars, NULL entries skipped).  Two launches; deterministic. */
#define DCS_GL_L1 1
#define DCS_GL_GRAD 2
#define DCS_GL_SSIM 4
#define DCS_GL_CA 8
#define DCS_GL_MSEC 16
typedef struct dcs_gl_job {
    const float* pred;
    const float* target;
    const float* source;
    const float* add0;
    const float* add1;
    float* grad;
    int32_t n_img, H, W, flags;
    float c_l1, c_grad, c_ssim, c_ca, c_mse, t_const, c_add0, c_add1;
} dcs_gl_job;
size_t dcs_gen_loss_fused_ws(const dcs_gl_job* jobs, int njobs);
int dcs_gen_loss_fused(const dcs_gl_job* jobs, int njobs, float ssim_data_range, float ca_sigma, float ca_min_w,
                       float ca_max_w, const float* bias, const float* coef, const float* coefx,
                       const float* const* extra, int nout, float* out, void* ws, size_t ws_bytes, void* stream);

/* Range-record arena: records (DCS_RANGE_PARTS floats each) inside [base, base + bytes) are zeroed
 * by the caller, in bulk, before each reuse of the arena; the producers that fold a record's maxima
 * then skip their own per-record memset.  Host-side registry of the calling process. */
int dcs_range_arena_register(const void* base, size_t bytes);
int dcs_range_arena_unregister(const void* base);

/* Partial maxima of |act(x * scale[n][c] + shift[n][c])| (or |x| when act == DCS_ACT_NONE and
 * scale == NULL) over an NHWC tensor of n_img images of `per_img` elements, C channels
 * innermost: DCS_RANGE_PARTS floats into parts, whose max bounds every value (the rng_a / rng_b
 * of an F16X3 pass).  per_img % 4 == 0, C % 4 == 0 with a prologue. */
int dcs_range_parts(const float* x, int n_img, int64_t per_img, int C, const float* scale,
                    const float* shift, int act, float* parts, void* stream);

/* ---- f16x3 window convolution: the residual-block 3x3 convs (modules/model.py:72-80) ----
 * A workgroup owns 256 consecutive pixels of one image (256 / W whole rows) x 128 output channels
 * and stages the (rows + 2) x (W + 2) source window once per 16-channel slice, split into hi / lo
 * fp16; the nine taps read MFMA fragments from it at a per-tap offset (csrc/conv_win.hip).
 *
 * dcs_pack_weights_h3: pre-split weights of a 3x3 conv, hi / lo fp16 planes [ncols][9 * C] in the
 * slice-major K order (k = (c / 16) * 144 + tap * 16 + c % 16), C = Cin for the forward (flip = 0) or
 * Cout for the data gradient over flipped taps (flip = 1); the values are scaled by 2^wexp[0]
 * (max |w| * 2^wexp < 2^15), written to *wexp on the device.  With flip = 1 out_hi / out_lo hold
 * 2 * ncols * 9 * Cout halves: the planes, then a tap-major copy (k = tap * Cout + c) that the data
 * gradient's ring reads.  scratch: DCS_RANGE_PARTS floats (dcs_pack_weights_h3_scratch_size bytes).
 * dcs_conv3_win_ok(d, dgrad): 1 if d is a geometry these passes cover: dgrad = 0, the forward of a
 * 3x3 stride-1 pad-1 conv (d as for dcs_conv_rows_in_stats); dgrad = 1, the padded-grid data gradient
 * (d as for dcs_conv_dgrad_reflect); both with mma = DCS_MMA_F16X3 and rng_a set, contiguous NHWC,
 * W <= 128, 256 % W == 0, H % (256 / W) == 0, Cs % 16 == 0, Co % 128 == 0.
 * dcs_conv3_win_in_stats: forward + IN statistics partials (as dcs_conv_rows_in_stats; parts = NULL
 * for none; *nchunk = H * W / 256).
 * dcs_conv_dgrad_reflect_win: the data gradient of a ReflectionPad2d(1) + 3x3 conv
 * (dcs_conv_dgrad_reflect's contract, plus the pre-split flipped weights): the interior by the
 * window pass (+ addend), the padded grid's one-pixel ring into ring (dcs_conv_dgrad_reflect_ring_size
 * bytes, any allocation) and folded onto dx's border; w_hi / w_lo: a flip = 1 pack with ncols == d->Co.
 * The ring: with Cs == 256 and Co % 256 == 0 one GEMM per ring segment and tap over the pack's tap-major
 * copy (csrc/conv_win.hip ring16_kernel: three ring
 * copies summed in tap order, independent of the batch), otherwise the rows pass over wpack (fp32
 * kind 1 | DCS_PACK_KSLICE with its range record). */
size_t dcs_pack_weights_h3_scratch_size(void);
int dcs_pack_weights_h3(const float* w, int Cout, int Cin, int flip, int ncols, void* out_hi, void* out_lo,
                        float* scratch, int* wexp, void* stream);
int dcs_conv3_win_ok(const dcs_conv_desc* d, int dgrad);
int dcs_conv3_win_in_stats(const dcs_conv_desc* d, const float* src, const void* w_hi, const void* w_lo,
                           const int* wexp, float* out, void* parts, size_t parts_bytes, int* nchunk, void* stream);
int dcs_conv_dgrad_reflect_win(const dcs_conv_desc* d, const float* dy, const float* wpack, const void* w_hi,
                               const void* w_lo, const int* wexp, const float* addend, float* dx, float* ring,
                               void* stream);
/* ---- f16x3 window convolution: the Generator's up-convolutions (modules/model.py:112-120) ----
 * nearest-x2 upsample + 3x3 zero-pad-1 conv as four 2x2 phase convolutions of the low-resolution
 * source (csrc/conv_subpix.hip): a workgroup owns 256 source pixels x 128 virtual columns (one column
 * phase, a 64-channel block, both row phases) and stages the source window once per 16-channel slice.
 * dcs_pack_subpix_h3: the phase weights (sums of the 3x3 taps that land on one source pixel) pre-split
 * into hi / lo fp16 planes, scaled by 2^wexp[0] of their own range; scratch: DCS_RANGE_PARTS floats.
 * kind 0: [4 Cout][4 Cin] (row = ((px * Cout / 64 + co / 64) * 2 + py) * 64 + co % 64, k = (c / 16) * 64 +
 * (u * 2 + t) * 16 + c % 16 for source offset (u, t)); Cout % 64 == 0, Cin % 16 == 0.  kind 1: the
 * transposed phase weights of the data gradient [Cin][16 Cout] (row = input channel, k = ((py * 2 + px) *
 * Cout / 16 + co / 16) * 64 + ((1 - u) * 2 + (1 - t)) * 16 + co % 16); Cout % 16 == 0, Cin % 128 == 0.
 * kinds 2 and 3: the stride-2 3x3 convolution's taps in kind 0's layout over dx's parity classes (its
 * data gradient, [4 Cin][4 Cout]; Cin % 64 == 0, Cout % 16 == 0) and in kind 1's layout over the source's
 * parity classes (its forward, [Cout][16 Cin]; Cout % 128 == 0, Cin % 16 == 0), zero where no tap lands;
 * kinds 5 and 4: the same for a 4x4 stride-2 convolution (w [Cout][Cin][4][4]).
 * dcs_subpix_win_ok(d): 1 if d is a sub-pixel rows descriptor (parity 2, as the rows pass takes it:
 * up = 1, Ho = 2 Hs) these kernels cover (contiguous NHWC, Cs % 16 == 0, Co % 64 == 0, min(Ws, 128)
 * dividing 256 and Ws, Hs % (256 / min(Ws, 128)) == 0, f16x3 / f16 with rng_a set, no prologue).
 * dcs_subpix_win: forward (+ IN statistics partials as dcs_conv_rows_in_stats when parts != NULL,
 * dcs_subpix_win_parts_size bytes; *nchunk = 4 x tiles per image). */
int dcs_pack_subpix_h3(const float* w, int Cout, int Cin, int kind, void* out_hi, void* out_lo, float* scratch,
                       int* wexp, void* stream);
int dcs_subpix_win_ok(const dcs_conv_desc* d);
size_t dcs_subpix_win_parts_size(const dcs_conv_desc* d);
int dcs_subpix_win(const dcs_conv_desc* d, const float* src, const void* w_hi, const void* w_lo, const int* wexp,
                   float* out, void* parts, size_t parts_bytes, int* nchunk, void* stream);
/* The data gradient of the same up-convolution (the adjoint: per phase a 2x2 conv of dy's phase sub-grid
 * with the transposed phase weights, dcs_pack_subpix_h3 with dgrad = 1).  d: the descriptor the rows pass
 * takes for it (source dy [N][Hs][Ws][Cs] contiguous, KH = KW = 4, stride 2, pt = pl = 1, zero pad, Ho = Hs / 2,
 * Wo = Ws / 2, Co = input channels of the forward, rng_a = dy's range record); dcs_subpix_win_dgrad_ok
 * checks it (Co % 128 == 0, min(Wo, 128) dividing 256 and Wo, Ho % (256 / min(Wo, 128)) == 0). */
int dcs_subpix_win_dgrad_ok(const dcs_conv_desc* d);
int dcs_subpix_win_dgrad(const dcs_conv_desc* d, const float* dy, const void* w_hi, const void* w_lo, const int* wexp,
                         float* dx, void* stream);
/* The down-convolutions (stride-2 3x3 zero-pad-1, modules/model.py:100-106) and the PatchGAN's stride-2
 * 4x4 zero-pad-1 layers (modules/model.py:118-131; every class offset a tap) on the same two kernels: the
 * forward as a sum over the source's four parity classes of <= 2x2 convolutions of the class sub-grids
 * (the sub-pixel data gradient's kernel; + IN statistics partials when parts != NULL,
 * dcs_stride2_win_parts_size bytes, *nchunk = tiles per image), the data gradient as four <= 2x2 phase
 * convolutions of dy onto dx's parity classes (the sub-pixel forward's kernel); the (class, offset) pairs
 * no tap reaches are skipped.  d: the rows pass's descriptor (parity 0: forward, Hs = 2 Ho, Co % 128 == 0;
 * parity 1: data gradient, Ho = 2 Hs, Co % 64 == 0), planes from dcs_pack_subpix_h3 kind 3 / 2 (3x3) or
 * 4 / 5 (4x4).  The forward takes the rows pass's prologue (d.pro_act AFFINE / RELU / LRELU with
 * pro_scale / pro_shift [N][Cs], Cs <= 512): a = act(y * scale + shift) staged, zero in the padding. */
/* Either data gradient (subpixel = 1: dcs_subpix_win_dgrad's descriptor and planes; 0: dcs_stride2_win's
 * parity-1 descriptor and planes) with the InstanceNorm backward's partial sums of its output fused, for
 * dx = da of a layer a = act(InstanceNorm(y)) (the down-convs' and up2's inputs): per (chunk, channel)
 * sum g and sum g * xhat, g = da * act'(xhat), xhat = y * scale + shift, into parts (Sum2 {float a, b}
 * [N][*nchunk][Co], dcs_phase_win_dgrad_inbwd_parts_size bytes) for dcs_in_act_backward_parts;
 * act DCS_ACT_AFFINE / _RELU / _LRELU, y NHWC like dx. */
size_t dcs_phase_win_dgrad_inbwd_parts_size(const dcs_conv_desc* d, int subpixel);
int dcs_phase_win_dgrad_inbwd(const dcs_conv_desc* d, int subpixel, const float* dy, const void* w_hi,
                              const void* w_lo, const int* wexp, float* dx, const float* y, const float* scale,
                              const float* shift, int act, void* parts, size_t parts_bytes, int* nchunk,
                              void* stream);
int dcs_stride2_win_ok(const dcs_conv_desc* d);
size_t dcs_stride2_win_parts_size(const dcs_conv_desc* d);
int dcs_stride2_win(const dcs_conv_desc* d, const float* src, const float* pro_scale, const float* pro_shift,
                    const void* w_hi, const void* w_lo, const int* wexp, float* out, void* parts, size_t parts_bytes,
                    int* nchunk, void* stream);
/* The same data gradient dx = da of a layer a = act(InstanceNorm(y)) (the first conv of a residual
 * block, modules/model.py:74-76), with the InstanceNorm backward's partial sums fused: the window
 * epilogue sums g = da * act'(xhat) and g * xhat (xhat = y * scale + shift) per (256-pixel tile,
 * channel) over the pixels the ring fold does not touch, and the fold sums its pixels with their final
 * values, into parts (Sum2 {float a, b} [N][*nchunk][Co], dcs_conv_dgrad_reflect_win_inbwd_parts_size
 * bytes) for dcs_in_act_backward_parts.  No addend; act DCS_ACT_AFFINE / _RELU / _LRELU; Co / 4
 * divides 256. */
size_t dcs_conv_dgrad_reflect_win_inbwd_parts_size(const dcs_conv_desc* d);
int dcs_conv_dgrad_reflect_win_inbwd(const dcs_conv_desc* d, const float* dy, const float* wpack, const void* w_hi,
                                     const void* w_lo, const int* wexp, float* dx, float* ring, const float* y,
                                     const float* scale, const float* shift, int act, void* parts, size_t parts_bytes,
                                     int* nchunk, void* stream);

/* Forward / data-gradient pass: out = gather(src) x B (+ bias, epilogue act). */
int dcs_conv_rows(const dcs_conv_desc* d, const float* src, const float* src2, const float* wpack,
                  const float* bias, const float* pro_scale, const float* pro_shift, float* out,
                  void* stream);

/* Forward pass with the InstanceNorm statistics of its output fused into the epilogue
 * (modules/model.py:94-111 — every conv that an InstanceNorm2d follows; aten convolution +
 * the statistics half of instance_norm): `out` as dcs_conv_rows, and per (row tile, channel) the
 * tile's count / mean / M2 / max / first argmax into `parts` (tiles never straddle images).
 * Needs parity 0 (or the sub-pixel forward, parity 2: per phase), Co > 4 and rows per image
 * % 128 == 0 (parts: dcs_conv_rows_in_stats_parts_size(d)
 * bytes; 0 = not applicable).  *nchunk receives the tiles per image, the `nchunk` of
 * dcs_in_stats_finish, which turns the partials into the scale / shift (and max / argmax) of
 * dcs_in_stats. */
size_t dcs_conv_rows_in_stats_parts_size(const dcs_conv_desc* d);
int dcs_conv_rows_in_stats(const dcs_conv_desc* d, const float* src, const float* src2, const float* wpack,
                           const float* bias, const float* pro_scale, const float* pro_shift, float* out, void* parts,
                           size_t parts_bytes, int* nchunk, void* stream);

/* Weight gradient: dw (OIHW) = sum_pixels dy^T x gather(x).  `d` describes the FORWARD conv
 * (source = x, output = dy).  ws must hold dcs_conv_wgrad_workspace_size(d) bytes. */
size_t dcs_conv_wgrad_workspace_size(const dcs_conv_desc* d);
int dcs_conv_wgrad(const dcs_conv_desc* d, const float* dy, const float* x, const float* x2,
                   const float* pro_scale, const float* pro_shift, float* dw, void* ws,
                   size_t ws_bytes, void* stream);

/* Data gradient of a 'same' K x K stride-1 convolution with ONE output channel (the Generator
 * head, modules/model.py:112: ReflectionPad(3) + Conv 7x7 64->1; aten convolution_backward
 * grad_input + reflection_pad2d_backward) onto its unpadded NHWC input:
 *   dx[n][y][x][c] = sum_{ty,tx} W[0][c][ty][tx] * sum_{(a,b) padding to (y,x)} dy[n][a-ty][b-tx]
 * dy: [N][H][W] (one channel); wk: the forward K-major pack ([(ty*K+tx)*C + c], dcs_pack_weights
 * kind 0, nmajor 0, ncols 1); dx: NHWC [N][H][W][C], C = 32 or 64; K = 3 or 7; 2*pad == K-1. */
int dcs_conv_dgrad_c1(const float* dy, int N, int H, int W, const float* wk, int C, int K, int pad, int pad_mode,
                      float* dx, void* stream);

/* Data gradient onto ONE input channel from C = 64 output channels: the image channel of the
 * Generator stem (modules/model.py:96-97, ReflectionPad(3) + Conv 7x7, stride 1) and the
 * PatchGAN's first layer (modules/model.py:121, Conv 4x4 stride 2 padding 1); aten
 * convolution_backward grad_input (+ reflection_pad2d_backward for the stem).  Two passes:
 *   z[q][t] = sum_c W[c][0][t] * dy[q][c]                                  (per dy pixel q)
 *   dx[n][y][x] = sum over padded positions (a,b) of (y,x) and taps t with (a-ty), (b-tx)
 *                 divisible by `stride` of z[n][(a-ty)/stride][(b-tx)/stride][t]
 * dy: NHWC [N][Hy][Wy][C]; wk[(ty*K+tx)*C + c] = W[c][0][ty][tx] (dcs_pack_weights kind 2, nmajor 0,
 * ncols 1, ci_count 1); (K, stride) = (7, 1) or (4, 2); pt/pl: top/left padding of pad_mode (reflect:
 * symmetric); dx: [N][H][W]; ws: dcs_conv_dgrad_to1_workspace_size(N, Hy, Wy, K) bytes. */
size_t dcs_conv_dgrad_to1_workspace_size(int N, int Hy, int Wy, int K);
int dcs_conv_dgrad_to1(const float* dy, int N, int Hy, int Wy, int C, const float* wk, int K, int stride, int pt,
                       int pl, int pad_mode, int H, int W, float* dx, void* ws, size_t ws_bytes, void* stream);

/* Pack up to 4 NCHW planes (x: [N][c1][H][W], x2: [N][c2][H][W] or NULL) into one NHWC
 * [N][H][W][4] tensor with zero channels after c1+c2 (c1 + c2 <= 4): the 4-channel layout the
 * vectorised stem convolution gathers (modules/model.py:94 input, trainer.py:451 concat). */
int dcs_pack_nhwc4(const float* x, int c1, const float* x2, int c2, int N, int H, int W, float* out,
                   float* rng,
                   void* stream);

/* Fold the gradient of a reflection-padded tensor back onto the tensor:
 * dx[n,i,j,c] = addend[n,i,j,c] + sum over padded positions mirroring to (i,j). */
/* Stride-1 data gradient of a ReflectionPad(1) + conv layer straight onto the unpadded grid
 * (modules/model.py:72-79 backward: aten convolution_backward + reflection_pad2d_backward, and
 * the residual add of the block when addend != NULL):
 *   dx[n][y][x][c] = addend[n][y][x][c] + sum over padded pixels (yp, xp) reflecting onto
 *                    (y, x) of (dy (*) flipped W)[n][yp][xp][c].
 * d describes the rows pass over the (H+2) x (W+2) padded grid exactly as for dcs_conv_rows
 * (pt = pl = KH-1, Ho = H+2, Wo = W+2, zero pad, stride 1).  The
 * conv epilogue writes interior pixels (plus the addend) into dx and the one-pixel ring into
 * ring (dcs_conv_dgrad_reflect_ring_size bytes); a small kernel then folds the ring in. */
size_t dcs_conv_dgrad_reflect_ring_size(const dcs_conv_desc* d);
int dcs_conv_dgrad_reflect(const dcs_conv_desc* d, const float* dy, const float* wpack, const float* addend,
                           float* dx, float* ring, void* stream);
int dcs_reflect_fold(const float* dxpad, const float* addend, float* dx, int N, int H, int W, int C,
                     int pad, void* stream);

/* Gradient of nearest x2 upsampling: dx[n,i,j,c] = sum_{a,b<2} dup[n,2i+a,2j+b,c]. */
int dcs_upsample2_grad(const float* dup, float* dx, int N, int H, int W, int C, void* stream);

/* ---- InstanceNorm2d(affine=False) (modules/model.py:61,94,97,110,124 → aten native_batch_norm) ---- */

/* Per-(n,c) statistics of an NHWC tensor: scale = 1/sqrt(var+eps), shift = -mean*scale
 * (so IN(x) = x*scale + shift), optional per-(n,c) max and argmax (pixel index) of x. */
size_t dcs_in_stats_workspace_size(int N, int HW, int C);
int dcs_in_stats(const float* x, int N, int HW, int C, float eps, float* scale, float* shift,
                 float* xmax, int32_t* xargmax, void* ws, size_t ws_bytes, void* stream);

/* The second half of dcs_in_stats over partials a producer wrote (dcs_conv_rows_in_stats):
 * parts [N][nchunk][C] chunk records, merged per (n,c) in a fixed order (deterministic). */
int dcs_in_stats_finish(const void* parts, int N, int C, int nchunk, float eps, float* scale, float* shift,
                        float* xmax, int32_t* xargmax, void* stream);

/* out = act(x*scale + shift) */
int dcs_in_apply(const float* x, const float* scale, const float* shift, float* out, int N, int HW,
                 int C, int act, float* rng,
                 void* stream);

/* Backward of a = act(IN(y)) given da: dy = scale*(g - mean(g) - xh*mean(g*xh)),
 * g = da*act'(xh), xh = y*scale+shift.  ws: dcs_in_stats_workspace_size(N,HW,C). */
int dcs_in_act_backward(const float* da, const float* y, const float* scale, const float* shift,
                        float* dy, int N, int HW, int C, int act, void* ws, size_t ws_bytes,
                        float* rng,
                        void* stream);
/* The same, its partial sums written by the producer of da (parts [N][nchunk][C] Sum2 records,
 * dcs_conv_dgrad_reflect_win_inbwd): merged per (n,c) in a fixed order, then applied.  ws: N*C*8 bytes. */
int dcs_in_act_backward_parts(const float* da, const float* y, const float* scale, const float* shift, float* dy,
                              int N, int HW, int C, int act, const void* parts, int nchunk, void* ws,
                              size_t ws_bytes, float* rng, void* stream);

/* ---- narrow-output convolutions (Co <= 4: Generator head, PatchGAN last layer, and the
 *      input-image gradients of the stem and the first PatchGAN layer) ---- */
int dcs_conv_rows_narrow(const dcs_conv_desc* d, const float* src, const float* src2,
                         const float* wpack, const float* bias, const float* pro_scale,
                         const float* pro_shift, float* out, void* stream);
/* The Generator head (modules/model.py:112: ReflectionPad2d(3) + Conv 7x7 64 -> 1 (+ bias) + Tanh) forward
 * in the fp16 operand modes, by tap projection on the MFMA pipe: z = a W (a = relu(src * pro_scale +
 * pro_shift) per (image, channel), W [64][49] from wpack = the narrow pack, K-major (tap * 64 + c) * ldb),
 * then a fixed-order 49-tap gather per output pixel.  d: the head's forward descriptor with pro_act =
 * DCS_ACT_RELU, epi_act DCS_ACT_NONE / _TANH, mma DCS_MMA_F16X3 / _F16 (dcs_head_fwd_proj_ok).  xmax:
 * [N][64] max of src per (image, channel) (dcs_in_stats_finish), for the operand scale.  out: [N][H][W]. */
int dcs_head_fwd_proj_ok(const dcs_conv_desc* d);
int dcs_head_fwd_proj(const dcs_conv_desc* d, const float* src, const float* wpack, const float* bias,
                      const float* pro_scale, const float* pro_shift, const float* xmax, float* out, void* stream);
/* The head's weight gradient in the same modes, by the transposed projection: dW[c][t] = sum_p a[p + off_t][c]
 * dy[p] as an MFMA GEMM (M = 64 channels, N = 49 taps, K = source columns) per workgroup band, the
 * workgroups' partials summed in a fixed order.  d, src, pro_scale, pro_shift, xmax as dcs_head_fwd_proj;
 * dy: [N][H][W] gradient at the conv output (before the bias); dw: [1][64][7][7] (OIHW).
 * ws: dcs_head_wgrad_proj_workspace_size(d) bytes. */
size_t dcs_head_wgrad_proj_workspace_size(const dcs_conv_desc* d);
int dcs_head_wgrad_proj(const dcs_conv_desc* d, const float* dy, const float* src, const float* pro_scale,
                        const float* pro_shift, const float* xmax, float* dw, void* ws, size_t ws_bytes,
                        void* stream);
/* The head's data gradient fused with the InstanceNorm + ReLU backward of its input (modules/model.py:110-112
 * backward) in the fp16 operand modes: da = the 7x7 reflect-pad-3 adjoint of dy_out onto 64 channels, on MFMA
 * (never written), then dy = IN-ReLU-backward(da) given y (the IN input, NHWC [N][H][W][64]) and its
 * per-(image, channel) scale / shift.  dy_out: [N][H][W] gradient at the head conv's output; wk: the weights
 * K-major, wk[(ty * 7 + tx) * 64 + c] = W[0][c][ty][tx].  act: DCS_ACT_RELU; mma: DCS_MMA_F16X3 / _F16;
 * H, W >= 8.  dy_rng: the range record of dy_out (dy_rng_n partial maxima, dcs_range_parts); rng: optional
 * range record of dy.  ws: dcs_head_dgrad_in_workspace_size(N, H, W) bytes. */
size_t dcs_head_dgrad_in_workspace_size(int N, int H, int W);
int dcs_head_dgrad_in(const float* dy_out, const float* dy_rng, int dy_rng_n, const float* wk, int N, int H, int W,
                      const float* y, const float* scale, const float* shift, int act, int mma, float* dy, void* ws,
                      size_t ws_bytes, float* rng, void* stream);
/* The Generator stem (modules/model.py:96-98: ReflectionPad2d(3) + Conv 7x7 cin -> 64 over the NHWC x 4
 * packed image, dcs_pack_nhwc4) forward in the f16x3 / f16 operand modes, on MFMA with the weights resident
 * in LDS.  d: the rows-pass descriptor of that conv (Cs = 4, pro_act / epi_act none, mma F16X3 / F16 with
 * both range records, ldb the packed weights' Kpad; dcs_stem_fwd_ok).  wpack: the rows pack (tap * 4 + c
 * K order).  parts (optional): per-(image, tile, channel) InstanceNorm partials for dcs_in_stats_finish
 * (dcs_stem_fwd_parts_size bytes; *nchunk receives the tiles per image). */
int dcs_stem_fwd_ok(const dcs_conv_desc* d);
size_t dcs_stem_fwd_parts_size(const dcs_conv_desc* d);
int dcs_stem_fwd(const dcs_conv_desc* d, const float* src, const float* wpack, float* out, void* parts,
                 size_t parts_bytes, int* nchunk, void* stream);
/* The stem's weight gradient in the same modes (rows pass over 64 output channels x 7 kernel-row blocks,
 * K = output pixels, on MFMA): d as for dcs_stem_fwd with cw = the weights' input channels (<= 4), rng_a
 * the range record of dy and rng_b that of the source; dw: [64][cw][7][7] (OIHW).
 * ws: dcs_stem_wgrad_workspace_size(d) bytes. */
int dcs_stem_wgrad_ok(const dcs_conv_desc* d);
size_t dcs_stem_wgrad_workspace_size(const dcs_conv_desc* d);
int dcs_stem_wgrad(const dcs_conv_desc* d, const float* dy, const float* src, float* dw, void* ws, size_t ws_bytes,
                   void* stream);
/* Pre-split fp16 planes of an N-major packed weight tensor for the f16x3 / f16 rows pass (dcs_conv_desc.b_h3):
 * out[r][0][k] = hi, out[r][1][k] = lo of wpack[r][k] * 2^e (fp16), e the operand exponent of the pack's range
 * record rng (dcs_pack_weights_r).  out: rows * 2 * ldb halves. */
int dcs_pack_split_h3(const float* wpack, int rows, int ldb, const float* rng, int rng_n, void* out, void* stream);
/* Every weight pack of a training step in two launches (instead of one or two small launches per pack).
 * A job is either a dcs_pack_weights_r pack (kind >= 0: w, Cout .. nmajor, out, rng as there; planes:
 * optional dcs_pack_split_h3 output of that pack, rows = ncols) or, with h3 = 1, a dcs_pack_weights_h3
 * pack (w, Cout, Cin, h3_flip, h3_ncols, h3_hi, h3_lo, h3_wexp, h3_scratch as there) or, with h3 = 2, a
 * dcs_pack_subpix_h3 pack (w, Cout, Cin, h3_flip = kind, h3_hi, h3_lo, h3_wexp, h3_scratch).  Results are
 * bit-identical to the per-pack calls.  jobs_dev: device copy of jobs[0 .. njobs) (the caller stages it;
 * jobs only supplies the host-side block counts); the b0 / b1 / p0 / p1 fields are filled here. */
typedef struct dcs_pack_job {
    const float* w;
    int32_t Cout, Cin, KH, KW, kind, ci_count, Kpad, ncols, nmajor, h3, h3_flip, h3_ncols;
    float* out;
    float* rng;
    void* planes;
    void* h3_hi;
    void* h3_lo;
    int32_t* h3_wexp;
    float* h3_scratch;
    int32_t b0, b1, p0, p1;  /* first block and block count of the job in the two launches (set by dcs_pack_plan) */
} dcs_pack_job;
/* Fills each job's block ranges and returns the grid sizes of the two launches (*g1, *g2). */
int dcs_pack_plan(dcs_pack_job* jobs, int njobs, int* g1, int* g2);
int dcs_pack_batch(const dcs_pack_job* jobs_dev, int njobs, int g1, int g2, void* stream);
size_t dcs_conv_wgrad_narrow_workspace_size(const dcs_conv_desc* d);
int dcs_conv_wgrad_narrow(const dcs_conv_desc* d, const float* dy, const float* x, const float* x2,
                          const float* pro_scale, const float* pro_shift, float* dw, void* ws,
                          size_t ws_bytes, void* stream);

/* ---- CBAM tail of ResidualBlockWithCBAM (modules/model.py:6-52, 83-87) ----
 * out = x + CBAM(IN(y)):  y is the raw conv2 output NHWC [N,H*W,C] with its InstanceNorm
 * coefficients (scale, shift) and the per-(n,c) max / argmax of y from dcs_in_stats.
 * w1: fc.0 [Cr][C], w2: fc.2 [C][Cr], wsa: [2][ksa][ksa] (spatial-attention conv, no bias).
 * Saved for backward: ca [N][C], sin_ [N][HW][2] (channel mean/max), sarg [N][HW] (argmax
 * channel), sa [N][HW]. */
int dcs_cbam_forward(const float* x, const float* y, const float* scale, const float* shift,
                     const float* ymax, const float* w1, const float* w2, const float* wsa,
                     int N, int H, int W, int C, int Cr, int ksa,
                     float* ca, float* sin_, int32_t* sarg, float* sa, float* out, float* rng,
                     void* stream);
size_t dcs_cbam_backward_workspace_size(int N, int H, int W, int C, int Cr, int ksa);
/* Given dout = dL/d(out): dy (gradient of the raw conv2 output y, InstanceNorm backward
 * included) and the gradients of w1, w2, wsa (overwritten).  The residual gradient (dout
 * itself, for x) is NOT added here. */
int dcs_cbam_backward(const float* dout, const float* y, const float* scale, const float* shift,
                      const float* ymax, const int32_t* yargmax, const float* w1, const float* w2,
                      const float* wsa, const float* ca, const float* sin_, const int32_t* sarg,
                      const float* sa, int N, int H, int W, int C, int Cr, int ksa, float* dy,
                      float* dw1, float* dw2, float* dwsa, void* ws, size_t ws_bytes, float* rng,
                      void* stream);

/* Global statistics of the batch-coupled losses over data-parallel ranks (SURVEY.md §8e
 * option ii; replaces the whole-batch reductions of modules/trainer.py:126-128 and :170-180
 * when the batch is sharded).  Phase functions: each leaves this shard's partial sums in a
 * caller buffer (red: double, histograms: uint32[512]) that the caller sums over ranks (one
 * all-reduce) before the next phase reads it.  All ranks then finish with the loss of the whole
 * batch; d loss / d pred of the local shard is multiplied by grad_scale (the world size, so
 * that the all-reduce-MEAN of parameter gradients equals the whole-batch gradient).  With one
 * rank and no reduction the result equals dcs_loss_contrast_region / _edge.  ws: the same
 * dcs_loss_workspace_size(N, H, W) buffer for every phase of one loss evaluation.
 *   region: partial -> sum red[0..6] -> finish
 *   edge:   partial -> sum red[0..4] -> for pass 0..3 { hist -> sum hist[0..511] -> select }
 *           -> topk -> sum red[5..8] -> finish                                           */
int dcs_loss_contrast_region_partial(const float* pred, const float* target, const float* source, int N, int H,
                                     int W, float threshold, double* red, void* ws, size_t ws_bytes, void* stream);
int dcs_loss_contrast_region_finish(const float* pred, int N, int H, int W, float weight, const double* red,
                                    float grad_scale, float* out, float* grad, void* ws, size_t ws_bytes,
                                    void* stream);
int dcs_loss_contrast_edge_partial(const float* pred, const float* target, int N, int H, int W, double* red,
                                   void* ws, size_t ws_bytes, void* stream);
int dcs_loss_contrast_edge_hist(int N, int H, int W, int pass, const double* red, uint32_t* hist, void* ws,
                                size_t ws_bytes, void* stream);
int dcs_loss_contrast_edge_select(int pass, const uint32_t* hist, void* ws, size_t ws_bytes, void* stream);
int dcs_loss_contrast_edge_topk(int N, int H, int W, double* red, void* ws, size_t ws_bytes, void* stream);
int dcs_loss_contrast_edge_finish(const float* pred, int N, int H, int W, const double* red, float grad_scale,
                                  float* out, float* grad, void* ws, size_t ws_bytes, void* stream);

/* ---- losses (modules/trainer.py:22-184, 347-351; pytorch_msssim.SSIM) ----
 * All take single-channel planes [N,1,H,W]; each writes the loss value to out[0] and the
 * gradient d(loss)/d(pred) (unscaled) to grad (may be NULL for value only). */
size_t dcs_loss_workspace_size(int N, int H, int W);
int dcs_loss_l1(const float* pred, const float* target, int64_t n, float* out, float* grad,
                void* ws, size_t ws_bytes, void* stream);
int dcs_loss_mse(const float* pred, const float* target, int64_t n, float* out, float* grad,
                 void* ws, size_t ws_bytes, void* stream);
int dcs_loss_mse_const(const float* pred, float target, int64_t n, float* out, float* grad,
                       void* ws, size_t ws_bytes, void* stream);
int dcs_loss_gradient(const float* pred, const float* target, int N, int H, int W, float* out,
                      float* grad, void* ws, size_t ws_bytes, void* stream);
int dcs_loss_contrast_attention(const float* pred, const float* target, const float* source, int N,
                                int H, int W, float sigma, float min_w, float max_w, int k,
                                float* out, float* grad, void* ws, size_t ws_bytes, void* stream);
int dcs_loss_contrast_region(const float* pred, const float* target, const float* source, int N,
                             int H, int W, float threshold, float weight, float* out, float* grad,
                             void* ws, size_t ws_bytes, void* stream);
int dcs_loss_contrast_edge(const float* pred, const float* target, int N, int H, int W, float* out,
                           float* grad, void* ws, size_t ws_bytes, void* stream);
int dcs_loss_ssim(const float* X, const float* Y, int N, int H, int W, float data_range,
                  int win, float sigma, float k1, float k2, float* out, float* grad, void* ws,
                  size_t ws_bytes, void* stream);

/* ---- optimizer (torch.optim.Adam, modules/trainer.py:360-362, 514, 520, 525) ----
 * One launch over a flat parameter buffer. */
int dcs_adam_step(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                  float beta2, float eps, float bias_c1, float bias_c2, void* stream);

/* ---- input pipeline (modules/preprocess.py:6-55, modules/mask_generator.py:11-347, as used by
 *      modules/dataset.py:109-181 for every training slice) ---- */

/* HU transform of N stored-pixel slices [N][H][W]: hu = f32(raw)*slope[n] + intercept[n]
 * (preprocess.py:45-46); img = [-1,1] image of clip(hu, hu_min, hu_max), soft-squeezed
 * (apply_soft_squeezing, preprocess.py:6-40, k = 10/sigma, threshold 0.9) when soft != 0, else
 * linear (preprocess.py:53).  raw_dtype: 0 int16, 1 uint16, 2 float32.  slope/intercept are
 * device arrays [N].  hu or img may be NULL (not written).  float32 op order as numpy. */
int dcs_hu_transform(const void* raw, int raw_dtype, const float* slope, const float* intercept, int N,
                     int H, int W, float hu_min, float hu_max, int soft, float sigma, float* hu,
                     float* img, void* stream);

/* Anatomical masks of N HU slices [N][H][W] (generate_anatomical_masks, 2-D path per slice):
 * lung (detect_lung), mediastinum (detect_mediastinum), bone (detect_bone), lung_vessel
 * (detect_lung_vessels).  Host arrays:
 *   thresholds[7] = {lung_lower, lung_upper, vessel_lower, vessel_upper, mediastinum_lower,
 *                    mediastinum_upper, bone_threshold}        (reference defaults -1000, -300,
 *                    -300, 600, -300, 450, 200)
 *   iparams[3]    = {min_size, border_margin, spine_start}     (64, 32, int(H*(1-0.25)))
 *   chan[4]       = output channel of {lung, mediastinum, bone, lung_vessel}, -1 = not wanted
 * out: float32 [N][nout][H][W] in {0,1} (the channel concat of dataset.py:135-158).
 * lung_in: optional device uint8 [N][H][W] binary lung mask used instead of detect_lung (the
 *   lung_mask argument of detect_mediastinum / detect_bone / detect_lung_vessels); NULL =
 *   computed from hu.
 * ws: dcs_masks_workspace_size(N, H, W) bytes.  H, W <= 1024.  Bit-exact with the reference. */
size_t dcs_masks_workspace_size(int N, int H, int W);
int dcs_anatomical_masks(const float* hu, const uint8_t* lung_in, int N, int H, int W, const float* thresholds,
                         const int32_t* iparams, const int32_t* chan, int nout, float* out, void* ws,
                         size_t ws_bytes, void* stream);

/* small utilities */
int dcs_scale_add(float* y, const float* x, float a, int64_t n, void* stream); /* y += a*x */
/* out = x * (*s) with s a device scalar (loss backward without a host sync) */
int dcs_scale_dev(const float* x, const float* s, float* out, int64_t n, void* stream);
/* dst[i][k] += src[i][k], k < n[i], for count tensors in one launch (host arrays of device
 * pointers; chunks of 64 tensors per launch). */
int dcs_multi_add(int count, const float* const* src, float* const* dst, const int64_t* n, void* stream);
/* dy = da * act'(y): relu/lrelu given the pre-activation y; tanh given the output y */
int dcs_act_backward(const float* da, const float* y, float* dy, int64_t n, int act, float* rng,
                     void* stream);
/* out[c] = sum_p x[p][c] (conv bias gradients) */
size_t dcs_channel_sum_workspace_size(int64_t P, int C);
int dcs_channel_sum(const float* x, int64_t P, int C, float* out, void* ws, size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DUCOSY_HIP_H */
