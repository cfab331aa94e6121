/* texbias.h -- C ABI of the MI355X (gfx950) k-space / spatial texture-filter library.
 *
 * This is the drop-in boundary for the hot path of yanielc/medical-vision-textural-bias:
 * the filters of source_code/filters_and_operators.py and the in-model layers of
 * source_code/stylization_layers.py, applied to batched [B][C][H][W][D] float32 volumes
 * resident in HBM.  Plain C types only (no torch), caller-owned device memory,
 * stream-ordered, no allocation or host synchronisation inside the launch functions
 * (graph-capturable).  Every function returns TB_OK (0) or a TB_ERR_* code.
 *
 * Reference interfaces each entry point replaces (file:line under the reference root):
 *   tb_kspace_filter_f32   Fourier.shift_fourier/inv_shift_fourier  filters_and_operators.py:594-632
 *                          + the k-space body of RandFourierDiskMaskd.__call__         :236-252
 *                          + RandPlaneWaves_ellipsoid.__call__                         :370-393
 *                          + WrapArtifact.__call__                                     :503-515
 *                          + GibbsNoise.__call__ / _apply_mask                         :663-705
 *                          + KSpaceSpikeNoise.__call__ / _set_spike                    :906-983
 *                          + GibbsNoiseLayer.forward / _apply_mask   stylization_layers.py:79-116
 *                          (one fused forward-FFT -> op program -> inverse-FFT round trip)
 *   tb_planes_closed_form_f32  RandPlaneWaves_ellipsoid.__call__ / KSpaceSpikeNoise._set_spike in
 *                          closed form (spike-only programs)                    :370-393, 966-983
 *   tb_salt_pepper_f32     SaltAndPepper.salt_and_pepper             filters_and_operators.py:465-482
 *   tb_minmax_f32          the x.max()/2, x.min()/2 of SaltAndPepper                   :476
 *   tb_disk_mask_f32       disk_mask.binary_mask_2d / binary_mask_3d                   :136-197
 *   tb_kspace_logabs_sum_f32   the default spike log-intensity 2.5*mean(log(|k|+1e-10)) :927-933, 1125-1131
 */
#ifndef TEXBIAS_H
#define TEXBIAS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TB_VERSION 1

/* error codes */
#define TB_OK 0
#define TB_ERR_INVALID_ARG 1
#define TB_ERR_UNSUPPORTED_SIZE 2 /* an axis longer than the direct-DFT fallback takes (10240) */
#define TB_ERR_HIP 3              /* a HIP runtime call failed; tb_last_hip_error() has the code */
#define TB_ERR_WORKSPACE 4        /* workspace smaller than tb_workspace_bytes() */

/* k-space op kinds (applied in program order to every half-spectrum coefficient) */
#define TB_OP_NONE 0
#define TB_OP_DISK 1  /* i[0]=int radius?, i[1]=inside_off, f[0]=fl32(r*r) or l=r*r (int)     */
#define TB_OP_GIBBS 2 /* l = integer threshold T4 on sum (2s-(n-1))^2 (float64 geometry)        */
#define TB_OP_LAYER 3 /* f[0] = alpha * max_dist (float32 geometry of GibbsNoiseLayer), or, when
                         l != 0, l = DEVICE address of a float alpha and f[1] = max_dist        */
#define TB_OP_WRAP 4  /* f[0] = alpha                                                           */
#define TB_OP_SPIKE 5 /* i[0..2] = UNSHIFTED (kh,kw,kd); f[0] = exp(log-intensity);
                         f[1] = phase override or NaN (keep own phase); f[2],f[3] = cos,sin(f[1]);
                         reserved = 1: same KSpaceSpikeNoise call as the previous SPIKE op (all
                         spikes of one call read the spectrum from before the call)          */
#define TB_OP_ZF 6    /* random k-space undersampling (RandZF, 50_reconstruction/reconGan/utils2.py:34-74):
                         coefficient (c, kh, kw, kd) (UNSHIFTED) is kept iff u > f[0] = p, with
                         u = (splitmix64(idx ^ l) >> 40) / 2^24, idx = ((c H + kh) i[1] + kw) i[2] + kd,
                         i[1] = W, i[2] = D, l = splitmix64(seed) (host); applied as (m(f) + m(-f)) / 2 */

#define TB_MAX_OPS 6
#define TB_MAX_BATCH 8 /* samples per launch group; larger batches are split by the library */

typedef struct tb_op {
  int32_t kind;
  int32_t chan; /* channel selector, -1 = all channels */
  int32_t i[3];
  int32_t reserved;
  int64_t l;
  float f[4];
} tb_op;

typedef struct tb_sample_ops {
  int32_t n; /* number of ops used */
  int32_t reserved[3];
  tb_op op[TB_MAX_OPS];
} tb_sample_ops;

/* transform geometry: spatial (H, W, D) after squeezing size-1 axes; D is contiguous */
typedef struct tb_plan tb_plan;

int tb_version(void);
const char* tb_error_string(int code);
int tb_last_hip_error(void);

/* Device id of the calling thread's current HIP device is used for the plan tables. */
int tb_plan_create(int H, int W, int D, tb_plan** out);
int tb_plan_destroy(tb_plan* plan);
/* Bytes of workspace needed for `bc` volume-channels (the half spectrum). */
size_t tb_workspace_bytes(const tb_plan* plan, int bc);
/* The FFT factorisation chosen for axis a (0=H,1=W,2=D): writes up to 8 radices, returns count. */
int tb_plan_radices(const tb_plan* plan, int axis, int* radices);

/*
 * y = Re(IFFT( ops_b,c( FFT(x) ) ))  for every sample b < B and channel c < C.
 *   x  : device, element (b,c,h,w,d) at x[(b*C+c)*xs[0] + h*xs[1] + w*xs[2] + d]
 *   y  : device, same indexing with ys[]; d in [D, D+y_pad) is written with 0
 *        (fuses the U-Net's D padding into the filter's store).  y may alias x.
 *   ws : device workspace of >= tb_workspace_bytes(plan, B*C) bytes
 *   ops: HOST array of B programs (copied into the launch arguments)
 *   minmax: optional DEVICE uint32[B][2] receiving the order-preserving keys of the
 *        per-sample min and max of y (the salt-and-pepper MIN/MAX), or NULL.
 */
int tb_kspace_filter_f32(const tb_plan* plan, const float* x, const int64_t* xs, float* y, const int64_t* ys,
                         int y_pad, void* ws, size_t ws_bytes, int B, int C, const tb_sample_ops* ops,
                         uint32_t* minmax, void* stream);

/*
 * The closed-form spike route on its own (SURVEY §8b's planes entry): RandPlaneWaves_ellipsoid.__call__
 * (filters_and_operators.py:370-393) and KSpaceSpikeNoise._set_spike (:966-983) for programs made only
 * of spikes that do not touch (no two at equal or conjugate frequencies in a shared channel):
 *   y = x + Re( sum_j Delta_j e^{2 pi i f_j . n / N} ) / N,   Delta_j = target_j(K(f_j)) - K(f_j)
 * Same arguments and results as tb_kspace_filter_f32 (which routes such programs here by itself);
 * TB_ERR_INVALID_ARG when a program is not of that form.  ws >= tb_workspace_bytes(plan, B * C).
 */
int tb_planes_closed_form_f32(const tb_plan* plan, const float* x, const int64_t* xs, float* y, const int64_t* ys,
                              int y_pad, void* ws, size_t ws_bytes, int B, int C, const tb_sample_ops* ops,
                              uint32_t* minmax, void* stream);

/*
 * Salt and pepper over B samples of `rows` rows of `len` floats (row pitch `ld`, sample pitch `sb`):
 *   cls = u <= thr[b][0] ? 1 (MIN) : u <= thr[b][1] ? 2 (MAX) : 0 (keep)
 *   y = cls==1 ? min_b/2 : cls==2 ? max_b/2 : x     (min_b/max_b from minmax keys)
 * u_in != NULL (parity mode): u is the caller's field, one value per voxel (the reference's
 *   torch.rand), classified exactly as above.
 * u_in == NULL: the device stream -- per segment of 256 voxels (TB_SAP_SEG), Philox4x32-10 (key seed,
 *   counter (sample << 44) ^ (segment << 20) | draw, stream `offset`) drives a geometric-gap walk over the changed
 *   voxels (gap = floor(log u / log(1 - thr[b][1]))) and each changed voxel's class (MIN with
 *   probability thr[b][0] / thr[b][1]): the same Bernoulli field at ~p of the RNG work.
 *   In place (x == y) only the changed voxels are stored; out of place y is a copy plus them.
 * cls (int8, same indexing as x) may be NULL.  thr is a HOST float[B][2].
 */
int tb_salt_pepper_f32(const float* x, float* y, int8_t* cls, const float* u_in, uint64_t seed, uint64_t offset,
                       const float* thr, const uint32_t* minmax, int B, int64_t rows, int len, int64_t ld,
                       int64_t sb, void* stream);

/* per-sample min/max keys of x (same row geometry as tb_salt_pepper_f32) into DEVICE uint32[B][2] */
int tb_minmax_f32(const float* x, uint32_t* minmax, int B, int64_t rows, int len, int64_t ld, int64_t sb,
                  void* stream);

/* decode an order-preserving key back to float (host helper) */
float tb_key_to_float(uint32_t key);

/* float32 binary disk/sphere mask of disk_mask (dim = 2 or 3 trailing axes), written for
 * `outer` repetitions of the n0 x n1 x n2 grid (n0 = 1 for dim 2).  int_r: compare in int64
 * against r2i; else float32 against r2f. */
int tb_disk_mask_f32(float* mask, int64_t outer, int n0, int n1, int n2, int int_r, int64_t r2i, float r2f,
                     int inside_off, void* stream);

/*
 * out[bc] = sum over the FULL spectrum of log(|FFT(x)| + 1e-10) (float64 accumulation),
 * after the first `n_pre` ops of each sample's program (the spike's own op excluded by the
 * caller).  Used for KSpaceSpikeNoise's default intensity 2.5*mean(...).  out: DEVICE double[B*C].
 */
int tb_kspace_logabs_sum_f32(const tb_plan* plan, const float* x, const int64_t* xs, void* ws, size_t ws_bytes,
                             int B, int C, const tb_sample_ops* ops, double* out, void* stream);

/*
 * Weight gradient of a 3x3x3 Conv3d / ConvTranspose3d (stride 1 or 2, padding `pad`), f32:
 *   dW[m][c][tz][ty][tx] = sum_n,z,y,x G[n][m][z][y][x] * X[n][c][s z+tz-pad][s y+ty-pad][s x+tx-pad]
 * G [N][M][Do][Ho][Wo] and X [N][Cc][Di][Hi][Wi] contiguous (device); dW [M][Cc][27] (device,
 * overwritten).  Conv3d: G = grad_out, X = input.  ConvTranspose3d: G = input, X = grad_out.
 * Replaces MIOpen's backward-weights for the U-Net's full-resolution layers (train step of
 * 10_scripts/20_Gibbs_filters/stylized_gibbs12p5.py:232-243).
 */
int tb_conv3d_wgrad_f32(const float* G, const float* X, float* dW, int N, int M, int Cc, int Do, int Ho, int Wo, int Di,
                        int Hi, int Wi, int stride, int pad, void* stream);

/*
 * The same weight gradient with a caller-owned workspace (device, `ws_bytes` from
 * tb_conv3d_wgrad_ws_bytes for the same sizes): the z-marching kernels then write one partial dW tile
 * per workgroup into `ws` and a reduction kernel sums them in workgroup order (deterministic) -- the
 * contended float atomics of tb_conv3d_wgrad_f32 cost up to 3/4 of those kernels' time.  `ws` NULL or
 * too small: tb_conv3d_wgrad_f32.  tb_conv3d_wgrad_ws_bytes returns 0 where no partial path exists.
 */
int64_t tb_conv3d_wgrad_ws_bytes(int N, int M, int Cc, int Do, int Ho, int Wo, int Di, int Hi, int Wi, int stride,
                                 int pad);
int tb_conv3d_wgrad_ws_f32(const float* G, const float* X, float* dW, int N, int M, int Cc, int Do, int Ho, int Wo,
                           int Di, int Hi, int Wi, int stride, int pad, void* ws, size_t ws_bytes, void* stream);

/*
 * The tiling tb_conv3d_wgrad_f32 chooses for these sizes, without launching anything (host only):
 * cfg[0] = SEG (64-column row segments staged per wave, 1..4), cfg[1] = TX (1: 16 input channels x
 * 27 tap accumulators; 3: (channel, tx) columns for <= 5 channels), cfg[2] = YB (output rows per
 * chunk), cfg[3] = chunks (work units), cfg[4] = LDS bytes per workgroup.  Same error codes.
 */
int tb_conv3d_wgrad_config(int N, int M, int Cc, int Do, int Ho, int Wo, int Di, int Hi, int Wi, int stride, int pad,
                           int64_t* cfg);

/*
 * Dice statistics of DiceLoss(sigmoid, squared_pred) (MONAI 0.5 formula, used by the reference's
 * train step stylized_gibbs12p5.py:201): for NC instances of S contiguous voxels of logits x and
 * target t, sums[nc] = {sum t p, sum t^2 (t), sum p^2 (p)} in float64 (DEVICE double[NC][3],
 * overwritten), p = sigmoid(x) if sigmoid else x.  The backward writes dx from the sums' gradients
 * g (DEVICE float[NC][3]).
 */
int tb_dice_sums_f32(const float* x, const float* t, double* sums, int64_t NC, int64_t S, int sigmoid, int squared,
                     void* stream);
/* The same sums without float atomics: float64 block partials in ws (tb_dice_sums_ws_bytes(NC, S) bytes of
 * device scratch) summed per instance in block order -- deterministic; two launches. */
size_t tb_dice_sums_ws_bytes(int64_t NC, int64_t S);
int tb_dice_sums_ws_f32(const float* x, const float* t, double* sums, int64_t NC, int64_t S, int sigmoid, int squared,
                        void* ws, size_t ws_bytes, void* stream);
/*
 * Dice METRIC statistics of the reference's evaluation loop (source_code/utils.py:313-411:
 * Activations(sigmoid=True) + AsDiscrete(threshold 0.5) then DiceMetric(include_background)):
 * sums[nc] = {sum t p, sum t, sum p} over S voxels with p = (sigmoid(x) >= 0.5) in {0, 1}.
 */
int tb_dice_metric_sums_f32(const float* x, const float* t, double* sums, int64_t NC, int64_t S, void* stream);
int tb_dice_sums_bwd_f32(const float* x, const float* t, const float* g, float* dx, int64_t NC, int64_t S, int sigmoid,
                         int squared, void* stream);
/*
 * DiceLoss's finalize from those sums (MONAI formula of the reference's DiceLoss, stylized_gibbs12p5.py:201):
 * f = 1 - (2 I + smooth_nr) / (G + P + smooth_dr) per instance (batch != 0: per channel, the sums added over
 * the NC / C samples); reduction 1: loss[0] = mean f, 2: loss[0] = sum f, 0: loss[i] = f[i] (DEVICE float).
 * The backward writes gsums [NC][3] (DEVICE float, the input of tb_dice_sums_bwd_f32) from the loss gradient
 * gloss (DEVICE float: one value, or one per f for reduction 0).  float64 arithmetic, one launch each.
 */
int tb_dice_loss_f32(const double* sums, float* loss, int64_t NC, int64_t C, int batch, int reduction, float smooth_nr,
                     float smooth_dr, void* stream);
int tb_dice_loss_bwd_f32(const double* sums, const float* gloss, float* gsums, int64_t NC, int64_t C, int batch,
                         int reduction, float smooth_nr, float smooth_dr, void* stream);

/*
 * out[c] = sum over n < N, s < S of x[n][c][s] (x contiguous [N][C][S], device; out DEVICE float[C],
 * overwritten): the bias gradient of a Conv3d / ConvTranspose3d, grad_out summed over (N, D, H, W)
 * -- replaces ATen's generic reduction in the U-Net backward (stylized_gibbs12p5.py:232-243).
 */
int tb_channel_sum_f32(const float* x, float* out, int64_t N, int64_t C, int64_t S, void* stream);
/* The same without float atomics: float64 block partials in ws (tb_channel_sum_ws_bytes(N, C, S) bytes of
 * device scratch) summed per channel in block order -- deterministic; two launches. */
size_t tb_channel_sum_ws_bytes(int64_t N, int64_t C, int64_t S);
int tb_channel_sum_ws_f32(const float* x, float* out, int64_t N, int64_t C, int64_t S, void* ws, size_t ws_bytes,
                          void* stream);

/*
 * Direct 3x3x3 convolution, stride 1, padding 1, for Cin, Cout <= 4 (the U-Net's full-resolution
 * 3 -> 3 ResidualUnit conv, where the implicit-GEMM library kernels run at ~1 TFLOP/s):
 *   y[n][co][z][h][w] = b[co] + sum w[co][ci][tz][ty][tx] x[n][ci][z+tz-1][h+ty-1][w+tx-1]
 * x [N][Cin][D][H][W], w [Cout][Cin][3][3][3], b [Cout] or NULL, y [N][Cout][D][H][W] (device,
 * contiguous); W <= 168.  The input gradient is the same call on grad_y with the flipped,
 * channel-transposed weights.
 */
int tb_conv3d_small_f32(const float* x, const float* w, const float* b, float* y, int N, int Cin, int Cout, int D,
                        int H, int W, void* stream);
/* The same with `add` (y's layout, or NULL) summed into the store: the U-Net's top ResidualUnit(3, 3,
 * conv_only) output conv(x) + x, and its input gradient dconv(dY) + dY, in one sweep. */
int tb_conv3d_small_add_f32(const float* x, const float* w, const float* b, const float* add, float* y, int N, int Cin,
                            int Cout, int D, int H, int W, void* stream);

/*
 * The U-Net's full-resolution stride-2 layers with few channels on one side (csrc/conv_up.hip; the
 * train step of 10_scripts/20_Gibbs_filters/stylized_gibbs12p5.py:192-243, MONAI UNet entry and exit):
 * tb_conv3d_s2_fewin_f32: out[n][m][o] = bias[m] + sum_{c < Cin, t} Wm[m][c][t] in[n][c][2 o + t - 1]
 *   (3x3x3, stride 2, padding 1; in [N][Cin][2 Do][2 Ho][2 Wo], out [N][Mout][Do][Ho][Wo]; Cin <= 4,
 *   Mout 16 or 32, 3 Wo <= 256), K = Wm as output-channel pairs: K[m / 2][c][t][m % 2].  Serves
 *   Conv3d(4 -> 16, s2)'s forward (Wm = its weight) and ConvTranspose3d(32 -> 3, s2)'s input gradient
 *   (in = dY, Wm = the transposed conv's [32][3][27] weight).
 * tb_convT3d_fewout_f32: ConvTranspose3d(Cin -> Mout, kernel 3, stride 2, padding 1, output_padding 1)
 *   forward, x [N][Cin][Di][Hi][Wi] -> y [N][Mout][2 Di][2 Hi][2 Wi], W = [Cin][Mout][3][3][3] as the
 *   module holds it; Mout <= 4, Cin <= 32, Wi % 4 == 0, Wi <= 128.  bias may be NULL for both.
 */
int tb_conv3d_s2_fewin_f32(const float* in, const float* K, const float* bias, float* out, int N, int Cin, int Mout,
                           int Do, int Ho, int Wo, void* stream);
int tb_convT3d_fewout_f32(const float* x, const float* W, const float* bias, float* y, int N, int Cin, int Mout, int Di,
                          int Hi, int Wi, void* stream);
/*
 * Conv3d(16 -> 16, kernel 3, stride 1, padding 1) forward on the f32 matrix cores (csrc/conv_up.hip):
 * x, y [N][16][D][H][W] (W % 16 == 0, W <= 128), weight [16][16][3][3][3], bias [16] or NULL.  The
 * U-Net's 16-channel full-resolution units (forward, and input gradient with W'[c][m][t] = W[m][c][26-t]).
 */
int tb_conv3d_fwd16_f32(const float* x, const float* W, const float* bias, float* y, int N, int D, int H, int Wd,
                        void* stream);
/* ... with `add` ([N][16][D][H][W] or NULL) summed into y: an identity-residual unit's input gradient
 * dconv(dZ) + dY in one sweep. */
int tb_conv3d_fwd16_add_f32(const float* x, const float* W, const float* bias, const float* add, float* y, int N, int D,
                            int H, int Wd, void* stream);
/* The layer's input gradient dX = conv(dY, W') (+ add) with W' = W[c][m][26 - t] read in the kernel from the
 * layer's own weight W [16][16][3][3][3] (no flipped copy); gy, dx [N][16][D][H][W]; add (or NULL) the same
 * per sample, add_sn floats apart (0: contiguous; a channel slice of a wider tensor otherwise). */
int tb_conv3d_fwd16_dgrad_f32(const float* gy, const float* W, const float* add, int64_t add_sn, float* dx, int N, int D,
                              int H, int Wd, void* stream);

/* ConvTranspose3d(64 -> 16, 3, stride 2, padding 1, output_padding 1) forward on the f32 matrix cores
 * (sub-pixel form, all 27 taps real): x [N][64][Di][Hi][Wi] -> y [N][16][2Di][2Hi][2Wi], weight
 * [64][16][3][3][3] as torch's module holds it, bias [16] or NULL; Wi % 4 == 0, Wi <= 64, x 16-B
 * aligned.  Replaces the col2im path torch.nn.functional.conv_transpose3d takes for the U-Net's up1
 * layer of the train step (10_scripts/20_Gibbs_filters/stylized_gibbs12p5.py:192-243, MONAI UNet). */
int tb_convT3d_mfma64_f32(const float* x, const float* W, const float* bias, float* y, int N, int Di, int Hi, int Wi,
                          void* stream);
/* The same for Cin = 32 or 64 (Cin -> 16); with a Conv3d(16 -> Cin, 3, s2, p1) layer's weight it is
 * that layer's input gradient (dX = conv_transpose3d(dY, W)). */
int tb_convT3d_mfma_f32(const float* x, const float* W, const float* bias, float* y, int N, int Cin, int Di, int Hi,
                        int Wi, void* stream);

/* Conv3d(C -> C, 3, stride 1, padding 1) forward for C = 32 or 64 on the f32 matrix cores (the input
 * channels split over the block's waves, partial tiles summed in LDS): x [N][C][D][H][W] -> y,
 * weight [C][C][3][3][3], bias [C] or NULL; W % 4 == 0, W <= 64 (C = 64: W <= 48), x 16-B aligned.
 * The input gradient of the layer is the same call with the flipped, transposed weight.  The U-Net's
 * 32- and 64-channel units of the train step (stylized_gibbs12p5.py:192-243, MONAI UNet). */
int tb_conv3d_mfma_f32(const float* x, const float* W, const float* bias, float* y, int N, int C, int D, int H, int Wd,
                       void* stream);
/* ... with `add` (y's layout or NULL) summed into y (as tb_conv3d_fwd16_add_f32). */
int tb_conv3d_mfma_add_f32(const float* x, const float* W, const float* bias, const float* add, float* y, int N, int C,
                           int D, int H, int Wd, void* stream);
/* The layer's input gradient with the flipped, transposed weight read in the kernel from W [C][C][3][3][3]
 * (as tb_conv3d_fwd16_dgrad_f32, `add` add_sn floats apart per sample). */
int tb_conv3d_mfma_dgrad_f32(const float* gy, const float* W, const float* add, int64_t add_sn, float* dx, int N, int C,
                             int D, int H, int Wd, void* stream);

/*
 * The U-Net's channel-deep convolutions as implicit GEMMs on the f32 matrix cores (csrc/conv_gemm.hip;
 * train step of 10_scripts/20_Gibbs_filters/stylized_gibbs12p5.py:192-243, MONAI UNet module tree
 * source_code/test.ipynb:754-1010 -- the stride-2 entries 16 -> 32 .. 64 -> 128, the 128/256-channel
 * bottom unit, the ConvTranspose3d ups and every one of their input gradients, which MIOpen/CK ran at
 * 23-51 TFLOP/s plus layout transposes).  x [N][Cin][D][H][Wd] with batch stride xsn (0: contiguous),
 * channel stride D H Wd; y likewise with batch stride ysn (0: contiguous); bias [M] or NULL; add (or
 * NULL) is summed into y (same layout as y, batch stride addsn; may alias y).  mode:
 *   TB_CG_CONV  (0): Conv3d(Cin -> M, ksize 3 (padding 1) or 1 (padding 0), stride 1 or 2), W [M][Cin][k^3];
 *   TB_CG_DGRAD (1): the input gradient of a stride-1 Conv3d(M -> Cin): x = dY [N][Cin][..], y = dX
 *                    [N][M][..], W = that layer's weight [Cin][M][k^3] (flipped and transposed inside);
 *   TB_CG_CONVT (2): ConvTranspose3d(Cin -> M, 3, stride 2, padding 1, output_padding 1) forward,
 *                    W [Cin][M][27] as the module holds it, y [N][M][2D][2H][2Wd] -- also the input
 *                    gradient of a stride-2 Conv3d(M -> Cin) with that layer's weight (x = dY, y = dX).
 * Cin % 4 == 0, W 16-B aligned, every tensor < 2^31 elements.  ws: device scratch of
 * tb_conv3d_gemm_workspace_bytes(...) bytes (packed weights, split-k partials; stream-ordered reuse).
 * tb_conv3d_gemm_config: cfg[0..5] = BM, BP, k slices, k per slice, blocks, positions (host only).
 */
#define TB_CG_CONV 0
#define TB_CG_DGRAD 1
#define TB_CG_CONVT 2
size_t tb_conv3d_gemm_workspace_bytes(int mode, int N, int Cin, int M, int D, int H, int Wd, int stride, int ksize);
int tb_conv3d_gemm_f32(int mode, const float* x, int64_t xsn, const float* W, const float* bias, const float* add,
                       int64_t addsn, float* y, int64_t ysn, int N, int Cin, int M, int D, int H, int Wd, int stride,
                       int ksize, void* ws, size_t ws_bytes, void* stream);
int tb_conv3d_gemm_config(int mode, int N, int Cin, int M, int D, int H, int Wd, int stride, int ksize, int64_t* cfg);

/*
 * Fused InstanceNorm3d(affine=False, eps) + PReLU(one weight a) over NC instances of S contiguous
 * voxels (x as [N][C][D][H][W], NC = N*C) -- the "ADN" block after every U-Net convolution
 * (MONAI Convolution, used by 10_scripts/20_Gibbs_filters/stylized_gibbs12p5.py:192-199).
 *   forward : y = prelu((x - mean) * rstd, a); stores mean[NC], rstd[NC] (biased var) for backward
 *   backward: dx (and, if dw != NULL, dw[0] = dL/da) from x, dy and the saved mean/rstd
 * prelu_w / dw are DEVICE pointers to one float.  ws: device scratch of
 * tb_instnorm_prelu_workspace_bytes(NC) bytes (reused per call, stream-ordered).
 */
size_t tb_instnorm_prelu_workspace_bytes(int64_t NC);
int tb_instnorm_prelu_fwd_f32(const float* x, float* y, float* mean, float* rstd, const float* prelu_w, int64_t NC,
                              int64_t S, float eps, void* ws, size_t ws_bytes, void* stream);
int tb_instnorm_prelu_bwd_f32(const float* x, const float* dy, const float* mean, const float* rstd,
                              const float* prelu_w, float* dx, float* dw, int64_t NC, int64_t S, void* ws,
                              size_t ws_bytes, void* stream);

/*
 * The same ADN block (InstanceNorm3d(affine=False) + PReLU) for the fused U-Net units of round 5:
 * per-sample batch strides (a channel slice of a wider tensor: *sn = floats between samples, 0 =
 * contiguous C S), the ResidualUnit's sum fused into the forward store (y = prelu(norm(x)) + res; res
 * may be NULL), and in the backward the preceding convolution's bias gradient dbias[c] = sum over n and
 * voxels of dx, taken in float64 from the backward statistics as -rstd mean(g z) sum(z) (the exact value
 * is zero: the norm removes a bias; NULL: not computed), dysum[c] = sum over n and voxels of dy (the
 * bias gradient of a residual convolution summed into the same output, out of the same sweep; NULL: not
 * computed), and the PReLU weight gradient dw (NULL: not computed).  No accumulator memsets and no float atomics: every block stores partial sums, reduced in
 * block order (by every apply block) -- results are
 * deterministic; two launches forward, two backward.  `counters`: DEVICE
 * uint32[tb_adn_counters(N, C)], zero before the first call, left zero by every call (one set per
 * stream); ws: tb_adn_workspace_bytes(N, C, S) bytes of device scratch.
 */
size_t tb_adn_workspace_bytes(int64_t N, int64_t C, int64_t S);
int64_t tb_adn_counters(int64_t N, int64_t C);
int tb_adn_fwd_f32(const float* x, int64_t xsn, float* y, int64_t ysn, const float* res, int64_t rsn, float* mean,
                   float* rstd, const float* prelu_w, int64_t N, int64_t C, int64_t S, float eps, void* ws,
                   size_t ws_bytes, uint32_t* counters, void* stream);
int tb_adn_bwd_f32(const float* x, int64_t xsn, const float* dy, int64_t dysn, float* dx, int64_t dxsn,
                   const float* mean, const float* rstd, const float* prelu_w, float* dw, float* dbias,
                   float* dysum, int64_t N, int64_t C, int64_t S, void* ws, size_t ws_bytes, uint32_t* counters,
                   void* stream);

/*
 * One Adam step over nt float32 tensors on the device, torch.optim.Adam semantics (L2 weight decay added
 * to the gradient; amsgrad: the denominator from the running maximum of exp_avg_sq), the reference's
 * optimizer (stylized_gibbs12p5.py:203-205: Adam(params, 1e-4, weight_decay=1e-5, amsgrad=True)).  The
 * pointer arrays are HOST arrays of DEVICE pointers; step[i] is tensor i's DEVICE float32 step count,
 * already incremented for this step (as torch's fused / capturable Adam keeps it); numel[i] (host) its
 * element count.  max_exp_avg_sq may be NULL without amsgrad.  Tensors are cut into 4096-element
 * chunks, up to 32 tensors per launch (csrc/optim.hip, k_adam).  Graph-capturable.
 */
int tb_adam_f32(int nt, float* const* param, const float* const* grad, float* const* exp_avg,
                float* const* exp_avg_sq, float* const* max_exp_avg_sq, const float* const* step,
                const int64_t* numel, double lr, double beta1, double beta2, double eps, double weight_decay,
                int amsgrad, void* stream);

/*
 * GPU-side BraTS preprocessing of B resident raw volumes img [B][C][H0][W0][D0] and
 * label maps lab [B][H0][W0][D0] (float class ids, as LoadImaged gives them; may be NULL when
 * out_lab is NULL), per sample b with params[b] drawn on the host:
 *   crop      out[.][i][j][k] = in[h0 + i][w0 + j][d0 + k]          RandSpatialCropd (MONAI 0.5)
 *   flip      bit 0/1/2 of `flip` mirrors spatial axis 0/1/2 inside the window   RandFlipd
 *   normalize (x - mean) / std over the window's nonzero voxels, per channel, std 0 -> 1
 *             (when `normalize`)                                   NormalizeIntensityd(nonzero, channel_wise)
 *   scale     x * scale  (scale = 1 + factor, or 1)                RandScaleIntensityd
 *   shift     x + shift on every voxel (or 0)                      RandShiftIntensityd
 * With `resample` = 1 the spatial part is instead one affine gather map per sample, built on the host
 * from Spacingd(pixdim, mode=("bilinear", "nearest")) -> Orientationd(axcodes) -> the crop ->
 * the flips (MONAI 0.5 semantics; …3modalities.py:156-161, val CenterSpatialCropd :186): output
 * voxel (i, j, k) samples the input at c = m[0..2] . (i, j, k) + m[3] (row a of the 3 x 4 map m
 * gives coordinate a), the image trilinearly and the label at the nearest voxel (round half to
 * even), both with border clamping (grid_sample padding_mode "border"); h0/w0/d0/flip are unused.
 * out [B][C][h][w][d]; out_lab [B][3][h][w][d] = (TC: 2|3, WT: 1|2|3, ET: 2) as 0/1 floats --
 * ConvertToMultiChannelBasedOnBratsClassesd, source_code/filters_and_operators.py:61-87.
 * Driver call site: 10_scripts/127_gibbs_spikes_wraparound_sap_OneChannel/
 * stylized_gibbs12p5_spikes15_wrap0p5_sap0p05_3modalities.py:151-170.  ws >= tb_brats_prep_workspace_bytes.
 */
typedef struct tb_prep_params {
  int h0, w0, d0; /* crop corner */
  int flip;       /* bit a: mirror spatial axis a */
  float scale;    /* 1 + factor, or 1 */
  float shift;    /* offset, or 0 */
  int normalize;  /* 1: NormalizeIntensity(nonzero=True, channel_wise=True) */
  int resample;   /* 1: spatial map m instead of crop + flip */
  float m[12];    /* resample: input coordinate a = m[4a] i + m[4a + 1] j + m[4a + 2] k + m[4a + 3] */
} tb_prep_params;
size_t tb_brats_prep_workspace_bytes(int B, int C);
int tb_brats_prep_f32(const float* img, const float* lab, int B, int C, int H0, int W0, int D0,
                      const tb_prep_params* params, int h, int w, int d, float* out, float* out_lab, void* ws,
                      size_t ws_bytes, void* stream);

/*
 * Compiled plans: slab shapes with a compile-time FFT plan (W x D = 240 x 155, 128 x 128) run passes
 * A and C on dedicated persistent kernels; enable = 0 forces the generic run-time-planned passes
 * (same results to rounding).  Default on; TEXBIAS_COMPILED_PLANS=0 in the environment turns it off.
 */
int tb_set_compiled_plans(int enable);

/*
 * Channel-volumes per pass A -> B -> C chain inside tb_kspace_filter_f32.  n > 0 runs the three
 * passes per chunk of n channel-volumes (the chunk's half spectrum is re-read by B and C from the
 * 256 MiB Infinity Cache rather than HBM), n = 0 runs each pass once over the whole batch group,
 * n < 0 restores the default (TEXBIAS_CHUNK_BC, else 0; chunking measured slower at C3).  Results
 * do not depend on n (bit-identical).
 */
int tb_set_chain_chunk(int n);

/*
 * Per-pass device timing for measurement: while enabled, every launch function records HIP
 * events around each of its kernels on the caller's stream.  tb_get_pass_times_ms synchronises
 * on them and returns the summed milliseconds per pass -- [0] slab forward (A), [1] k-space
 * pencil pass (B), [2] slab inverse (C), [3] salt-and-pepper / minmax -- and the launch counts,
 * then clears the record.  Disabled by default (no events, graph-capturable).
 */
int tb_set_pass_timing(int enable);
int tb_get_pass_times_ms(float* ms_sum4, int* count4);
/* Same record plus the summed ALGORITHMIC bytes per pass (each global input/output element of a
 * launch counted once; sparse salt-and-pepper counts 0), then clears it.  bytes4 may be NULL. */
int tb_get_pass_stats(float* ms_sum4, int* count4, double* bytes4);
/* Name of the kernel last timed in pass slot 0..3 ("" if none). */
const char* tb_pass_kernel(int slot);

/*
 * Band-limited plans: a program containing an all-channel low-pass (disk with inside_off = 0,
 * Gibbs, or a layer mask with host alpha) whose kept box is small runs the pruned passes A'/B'/C'
 * (one image read, one image write, the box spectrum in between) instead of the full-spectrum
 * passes; spikes outside the box are synthesised in the same store.  Same results to rounding.
 * Default on; TEXBIAS_BAND=0 in the environment turns it off.  Samples whose program is empty are
 * copied through unchanged (bit-identical, as the reference returns them untouched).
 */
int tb_set_band_plans(int enable);

/*
 * Spike-only programs (RandPlaneWaves_ellipsoid, KSpaceSpikeNoise: filters_and_operators.py:370-393,
 * 966-983) whose spikes do not touch (no two at equal or conjugate frequencies in a shared channel) run
 * in closed form, y = x + Re(sum_j Delta_j e^{2 pi i f_j.n/N}) / N with Delta_j = target_j(K(f_j)) - K(f_j):
 * one pass computing the coefficients K(f_j), one streaming add (12 B per voxel instead of a spectrum
 * round trip).  Same results to rounding.  Default on; TEXBIAS_POINT=0 in the environment turns it off.
 */
int tb_set_point_plans(int enable);

/*
 * Wrap-only programs (WrapArtifact, filters_and_operators.py:503-515) on shapes with even H and W take
 * the separable route: the mask is a product of symmetric 1-D masks, so y = T_h T_w T_d x with 2-tap
 * circulants on the even axes and, for odd D (D + pad <= 256), a dense D-point circulant applied as a
 * split-f16 matrix product -- one image read and one write, no spectrum.  Same results to rounding.
 * Default on; TEXBIAS_WRAP=0 in the environment turns it off.
 */
int tb_set_wrap_plans(int enable);

/*
 * Full-spectrum route (Fourier.shift_fourier / inv_shift_fourier, filters_and_operators.py:594-632)
 * on shapes with a half-unit plan (240 x 240 x 155): passes A and C run per (slab, row parity) --
 * the W transform split at its last radix-2 step, two workgroups per CU -- and pass B finishes the
 * W transform with the butterfly (split spectrum in the workspace).  Same results to rounding.
 * Default on; TEXBIAS_HALF=0 in the environment or tb_set_half_units(0): whole-slab passes.
 */
int tb_set_half_units(int enable);

/*
 * Pass C' of the band-limited plans synthesises the image on the f16 matrix cores in split
 * precision (table and V each as an f16 hi/lo pair, three products, f32 accumulation; agrees with
 * the f32 synthesis to a few 1e-7 of max |y|) whenever the launch's band columns plus all of its
 * samples' out-of-box spike points number at most 32; otherwise, or after tb_set_band_inv16(0)
 * (TEXBIAS_INV16=0 in the environment), the f32 MFMA synthesis.  Default on.
 */
int tb_set_band_inv16(int enable);

#ifdef __cplusplus
}
#endif
#endif /* TEXBIAS_H */
