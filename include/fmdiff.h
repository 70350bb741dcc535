/*
 * fmdiff: MI355X-native (gfx950 / CDNA4) kernels for the flow-matching /
 * diffusion UNet train + sample hot path.  C ABI, plain pointers and sizes.
 *
 * Ownership: every buffer (activations, weights, workspaces) is allocated by
 * the caller (PyTorch's caching allocator) and passed in; the library
 * allocates nothing.  Errors: every entry point returns 0 on success, a
 * positive hipError_t, or a negative argument-validation code; no exception
 * crosses the ABI.  Threading: kernels are stateless and launch on the
 * caller's hipStream_t.
 *
 * Layouts: activations NHWC bf16 ("pixels x channels"); conv weights bf16
 * [K][ks*ks][C] (forward) -- the fp32 master copy stays in the reference's
 * [K][C][kh][kw] layout so state_dicts are drop-in.
 *
 * The reference has no native plugin API: its boundary is the Python module
 * surface.  Each entry point names the reference op(s) it replaces.
 */
#ifndef FMDIFF_H
#define FMDIFF_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* fmd_stream_t; /* hipStream_t */

/* ------------------------------------------------------------------ conv
 * Implicit-GEMM convolution on MFMA, replacing ConvND -> nn.Conv{2}d
 * (src/nn/ops/convolution.py:8-54), the GroupNorm+SiLU(+scale/shift) that
 * feeds it (src/nn/blocks/residual.py:95-117), nearest-x2 UpsampleND
 * (src/nn/ops/upsampling.py:27), DownsampleND stride 2 (upsampling.py:49-56),
 * the decoder torch.cat (src/models/unet/unet.py:322), the 1x1 skip conv and
 * residual add (residual.py:120).  The same kernel computes data gradients
 * (transposed gather) for the backward pass.
 */
typedef struct fmd_conv_desc {
  int32_t N, Hs, Ws;        /* stored input dims */
  int32_t C0, C1;           /* channels of src0 / src1 (virtual concat, C = C0 + C1) */
  int32_t Ho, Wo, K;        /* output dims / output channels */
  int32_t ks, stride, pad;  /* square kernel, stride, zero padding */
  int32_t upsample;         /* 1: logical input = nearest-x2 of the stored input */
  int32_t transposed;       /* 1: gather (o + pad - k) / stride  (data-gradient mode) */
  const void* src0;         /* bf16 NHWC [N][Hs][Ws][C0] */
  const void* src1;         /* bf16 NHWC [N][Hs][Ws][C1] or NULL */
  const float* pro_a;       /* [N][C] prologue affine x*a+b (GroupNorm fused), or NULL */
  const float* pro_b;
  int32_t pro_silu;         /* apply SiLU after the affine */
  const void* wgt;          /* bf16 [K][ks*ks][C] */
  const void* src2;         /* optional 1x1 second GEMM over the concat (src2 | src3): */
  const void* src3;         /*   bf16 [N][Ho][Wo][C2] and [N][Ho][Wo][C3] (ResBlock skip conv) */
  int32_t C2, C3;
  const void* wgt2;         /* bf16 [K][C2+C3] */
  const float* bias;        /* [K] or NULL */
  const float* bias2;       /* [K] or NULL (skip-conv bias, added too) */
  const float* bias_nc;     /* [N][K] per-sample bias (time-embedding add) or NULL */
  const void* resid;        /* bf16 [N][Ho][Wo][K] residual or NULL */
  void* out;                /* bf16 (or fp32 if out_f32) [N][Ho][Wo][K] */
  int32_t out_f32;
  int32_t accumulate;       /* out += result */
  float* stats;             /* slab [M/64][K][2] of per-64-pixel partial sums, or NULL; with splits > 1
                               [M/FMD_SPLIT_STATS_ROWS][K][2] (written by the split-K combine), or
                               [M/tickets_rows][K][2] when the split is combined inside the launch (tickets) */
  const void* ep_x0;        /* data-gradient epilogue: x = forward GN input at (p, c); if ep_a: */
                            /*   out *= silu'(ep_a*x+ep_b); stats become (sum out, sum out*x) */
  const void* ep_x1;
  int32_t ep_C0;
  const float* ep_a;
  const float* ep_b;
  float* ws;                /* split-K workspace fp32 [splits][M][K] */
  int32_t splits;
  int32_t force_generic;    /* 1: never take the halo-tiled 3x3 path (testing) */
  const void* wgt_tiled;    /* wgt re-tiled by fmd_tile_weights_halo (enables the halo path) */
  const void* wgt2_tiled;   /* wgt2 re-tiled likewise (T = 1) */
  int32_t Ds, Do;           /* 3-D problems (spatial_dims = 3, NDHWC): stored / output depth; 0 = 2-D.
                               Cubic kernel (ks^3 taps, wgt [K][ks^3][C]); implicit-GEMM path only */
  void* gout;               /* optional bf16 [N][Hs][Ws][C0+C1] (3-D: [N][Ds][Hs][Ws][C]): the prologue's output
                               G = SiLU(pro_a*x+pro_b) (or the affine alone), written once per element by the
                               halo path -- the weight gradient's operand, so the backward does not recompute
                               the GroupNorm+SiLU.  Requires pro_a, (C0+C1) % 32 == 0 and the halo path (fmd_conv
                               returns -9 otherwise); NULL = off */
  const float* fold_st0;    /* forward-only GroupNorm prologue folded in the halo kernel (2-D, csrc/conv_halo9.hip),
                               in place of pro_a / pro_b: each workgroup computes its sample's affine from the
                               producers' statistics slab of src0 [N*Hs*Ws/fold_rows0][C0][2] (and of src1), the
                               groups, eps, gamma, beta and the scale-shift rows -- gn_prep's fold, without its
                               launch.  fmd_conv returns -13 when the v9b halo kernel does not take the problem
                               (the caller folds with fmd_gn_prep instead).  NULL = off */
  int32_t fold_rows0;
  const float* fold_st1;
  int32_t fold_rows1;
  int32_t fold_G;
  float fold_eps;
  const float* fold_gamma;  /* [C0 + C1] or NULL */
  const float* fold_beta;
  const float* fold_emb;    /* scale-shift norm: [N][fold_emb_stride] scale | shift, or NULL */
  int32_t fold_emb_stride;
  int32_t* tickets;         /* split-K (splits > 1) combined inside the conv launch (2-D: the v9b halo kernel or the
                               implicit GEMM on whole tiles): [n_tickets] arrival counters, zero on entry and left
                               zero; d->ws holds the parts' fp32 tiles (same [splits][M][K] size) and the statistics
                               come from the conv epilogue, one row per tickets_rows pixels (64 on the halo kernel,
                               the wave's pixel range on the implicit GEMM).  fmd_conv returns -14 when the kernel
                               that takes the problem cannot combine it so or would write other rows (the caller then
                               runs the two-launch split).  NULL = the separate combine launch */
  int32_t n_tickets;
  int32_t tickets_rows;     /* pixels per statistics row the caller allocated for a ticketed conv with stats */
} fmd_conv_desc;

/* Dispatches 3x3 stride-1 forward-gather problems with >= 128 16x16 output tiles to the
 * halo-tiled kernel (csrc/conv_halo.hip), everything else to the implicit GEMM (csrc/conv.hip). */
int fmd_conv(const fmd_conv_desc* d, fmd_stream_t s);
/* Halo-tiled 3x3 stride-1 conv; returns 1 (nothing launched) when the problem does not qualify. */
int fmd_conv_halo(const fmd_conv_desc* d, fmd_stream_t s);
/* Split-K combine alone: d->out = sum of the d->splits fp32 slabs [splits][M][K] in d->ws + the conv epilogue
 * (bias, bias2, bias_nc, resid, ep_*, stats with FMD_SPLIT_STATS_ROWS-pixel rows).  Replaces nothing on its
 * own: it closes convolutions issued as several partial launches (3-D 3x3x3 convs as three depth-tap planes
 * of the 2-D halo kernel, ConvND 3-D path, src/nn/ops/convolution.py:36). */
int fmd_conv_combine(const fmd_conv_desc* d, fmd_stream_t s);
/* GroupNorm-backward apply fused as a conv epilogue (fmd_conv_gn_apply):
 * dx = conv(d) + P*dz + Q*x + R (+ dx if acc), x/dx split over two concat sources at C0. */
typedef struct fmd_gn_apply_desc {
  const void* dz;           /* bf16 [M][C] (C = the conv's K) */
  const void* x0;           /* bf16 [M][C0] forward GroupNorm input */
  const void* x1;           /* bf16 [M][C - C0] or NULL */
  int32_t C0;
  const float* P;           /* [N][C] */
  const float* Q;
  const float* R;
  void* dx0;                /* bf16 [M][C0] */
  int32_t acc0;
  void* dx1;                /* bf16 [M][C - C0] or NULL */
  int32_t acc1;
} fmd_gn_apply_desc;
/* The ResBlock skip-conv data gradient fused into the GroupNorm backward of the block input
 * (replaces conv(dy, W_skip^T) + fmd_gn_bwd_apply(extra = that)). */
int fmd_conv_gn_apply(const fmd_conv_desc* d, const fmd_gn_apply_desc* g, fmd_stream_t s);

/* GroupNorm forward of a split-K conv's output, fused into its split-K combine (fmd_conv_gn).  For each (n, c):
 * out = conv result (bf16, as fmd_conv writes it); then per (n, group) mean / rstd of out, a = rstd*gamma,
 * b = beta - mean*a (emb_mode 1: a *= 1 + emb[n][c], b = b*(1 + emb[n][c]) + emb[n][K + c]) and the materialised
 * t = SiLU(a*out + b) (silu = 0: the affine alone) -- the outputs of fmd_gn_fused_apply on out. */
typedef struct fmd_gn_out_desc {
  int32_t G;                /* groups */
  float eps;
  const float* gamma;       /* [K] or NULL */
  const float* beta;        /* [K] or NULL */
  const float* emb;         /* [N][emb_stride] scale | shift (emb_mode 1) or NULL */
  int32_t emb_stride, emb_mode, silu;
  float* a;                 /* [N][K] */
  float* b;                 /* [N][K] */
  float* mean_rstd;         /* [N][G][2] */
  void* t;                  /* bf16 [N][Ho][Wo][K] */
} fmd_gn_out_desc;
/* fmd_conv with d->splits > 1 whose combine also produces the GroupNorm of the output (one workgroup per
 * (image, whole groups of max(CB = 4 or fmd_conv_gn_set_block_channels, C/G) channels): the group statistics close inside it).  Requires K % 64 == 0, 64 % (K/G) == 0, no
 * d->stats / out_f32 / accumulate / ep_*.  Replaces fmd_conv + fmd_gn_fused_apply on the small levels
 * (src/nn/blocks/residual.py:71-76 conv1 -> out_layers GroupNorm + SiLU). */
int fmd_conv_gn(const fmd_conv_desc* d, const fmd_gn_out_desc* g, fmd_stream_t s);

/* Input channels per halo-kernel chunk (csrc/conv_halo.hip). */
#define FMD_SPLIT_STATS_ROWS 16   /* pixels per statistics row of a split-K conv */
/* Fewest workgroups (16x16 tiles x cout tiles x split-K chunks) a 2-D problem needs to take the halo conv
 * (default 32; fewer go to the implicit GEMM).  The Python side applies its tuning table's HALO_MIN_WG through it
 * (fmdiff/runtime/tuning.py); the host's halo_splits mirror reads the same table entry. */
int fmd_halo_set_min_workgroups(int32_t n);
/* Halo-conv grids with fewer workgroups than n (16-row tiles x cout tiles x splits; default 1024) run 8-row tiles
 * instead (twice the workgroups: the 128^2 / 64^2 levels would otherwise be one lock-step round); 0 = never.  A
 * tuning hook (tuning table HALO_TH8_MAX_WG). */
int fmd_halo_set_th8_max_workgroups(int32_t n);
/* 8-row grids (tiles x splits) with fewer workgroups than n (default 512) run 4-row tiles instead (plain 2-D 3x3:
 * the latent UNet's 32^2 convs would otherwise fill half the CUs); 0 = never.  Tuning table HALO_TH4_MAX_WG. */
int fmd_halo_set_th4_max_workgroups(int32_t n);
/* Fewest channels per combine block of fmd_conv_gn (4, 8, 16, 32 or 64; default 4):
 * a block owns max(cb, K / G) channels = whole groups.  Returns -1 for any other value.  A tuning hook; the host's
 * conv_gn_eligible mirror reads ops.CONV_GN_CB. */
int fmd_conv_gn_set_block_channels(int32_t cb);
#define FMD_HALO_BK 32
/* [K][T][C] bf16 kernel weights -> the halo kernel's per-(cout tile, FMD_HALO_BK-channel chunk, tap) 8 KiB tiles. */
int64_t fmd_halo_tiled_size(int32_t K, int32_t T, int32_t C);
int fmd_tile_weights_halo(const void* w, int32_t K, int32_t T, int32_t C, void* out, fmd_stream_t s);
/* Stride-2 pad-1 convs (3x3, or the 4x4 data gradient of conv3x3(nearest_x2(x))) as a 2x2 conv over the
 * space-to-depth view of the input (plane (a, b) = pixels (2y + a, 2x + b), staged from the full-resolution NHWC
 * tensor) on the halo kernel (csrc/conv_halo9.hip).  Replaces the implicit GEMM of DownsampleND's conv
 * (src/nn/ops/upsampling.py:49-56) and the data gradient of UpsampleND's conv (upsampling.py:27-29).  Needs
 * d->wgt_tiled from fmd_s2d_tile_weights, Hs = 2 Ho, Ws = 2 Wo, Ho and Wo multiples of 16, (C0 + C1) % 32 == 0,
 * K % 128 == 0, >= 128 output tiles; d->accumulate adds into d->out.  3-D (d->Ds = 2 d->Do, stride 2 in depth too;
 * weights from fmd_s2d_tile_weights_nd with dims 3): the depth taps run as chunks over full-resolution slices
 * 2z + kz - 1 (Conv3d of DownsampleND; the 4x4x4 data gradient of UpsampleND's Conv3d).  Returns 1 when the problem
 * does not qualify. */
int fmd_conv_s2d(const fmd_conv_desc* d, fmd_stream_t s);
/* The data gradient of a stride-2 pad-1 3x3 conv (the transposed gather of DownsampleND's conv,
 * src/nn/ops/upsampling.py:49-56) as a stride-1 2x2 conv from the low-resolution gradient onto the depth-to-space
 * view of the output (4 pixel classes x K channels, one class per 128-channel tile) on the halo kernel.  d as for
 * fmd_conv with transposed = 1: Ho = 2 Hs, Wo = 2 Ws, Hs and Ws multiples of 16, (C0 + C1) % 32 == 0, K % 128 == 0,
 * no prologue; d->wgt_tiled from fmd_s2d_tile_weights mode 2; d->accumulate adds into d->out.  3-D (d->Do = 2 d->Ds,
 * weights from fmd_s2d_tile_weights_nd with dims 3): 8 output classes (depth parity, a, b), the gradient slices z and
 * z + 1 as chunks.  Returns 1 when the problem does not qualify. */
int fmd_conv_d2s(const fmd_conv_desc* d, fmd_stream_t s);
/* fp32 reference-layout conv weight [K][C][ks][ks] -> the halo tiles of fmd_conv_s2d / fmd_conv_d2s.  mode 0: the
 * stride-2 forward (rows K, ks 3 or 4); mode 1: the 4x4 data gradient of a 3x3 conv on a nearest-x2 input
 * (rows C, inner channels K, ks 3); mode 2: the stride-2 3x3 data gradient (rows 4C class-major, C % 128 == 0,
 * inner K).  The inner channel count must be a multiple of 32. */
int64_t fmd_s2d_tiled_size(int32_t K, int32_t C, int32_t mode);
int fmd_s2d_tile_weights(const float* w, int32_t K, int32_t C, int32_t ks, int32_t mode, void* out, fmd_stream_t s);
/* The same for 2-D (dims 2, as above) or 3-D (dims 3) masters: [K][C][3][3][3] fp32 -> the 3-D tiles of
 * fmd_conv_s2d / fmd_conv_d2s (mode 0: 3 depth taps x the 2-D chunks; mode 1: the 4 folded depth taps; mode 2: rows
 * 8C class-major, 2 depth offsets). */
int64_t fmd_s2d_tiled_size_nd(int32_t K, int32_t C, int32_t mode, int32_t ks, int32_t dims);
int fmd_s2d_tile_weights_nd(const float* w, int32_t K, int32_t C, int32_t ks, int32_t mode, int32_t dims, void* out,
                            fmd_stream_t s);

/* Small-level conv in ONE launch (csrc/conv_small.hip): the sampler's low-resolution levels, where the split-K
 * implicit GEMM needed a combine launch and a GroupNorm launch beside every conv.  A workgroup owns up to 64 output
 * pixels (64-pixel blocks of one image, or whole images when Ho*Wo < 64) x 16 output channels and the FULL reduction:
 * the input rows its taps read (all C = C0 + C1 channels) are staged once in LDS with the GroupNorm affine
 * (+ scale/shift) + SiLU applied -- the affine folded in-kernel from the producers' statistics slabs -- and eight
 * waves split the 32-channel chunks, combining in LDS in a fixed order.  Replaces, per conv, ResBlockND's
 * GroupNorm(+scale/shift)+SiLU -> ConvND 3x3 (src/nn/blocks/residual.py:84-120, normalization.py:11-19,
 * convolution.py:8-54) with the time-embedding add, the 1x1 skip conv + residual add (residual.py:77-82, 120),
 * DownsampleND's stride-2 conv and UpsampleND's nearest-x2 + conv (upsampling.py:8-62), and emits the per-channel
 * statistics the next GroupNorm folds.  Forward only (no saved affine for a backward). */
typedef struct fmd_conv_small_desc {
  int32_t N, Hs, Ws, C0, C1; /* input bf16 NHWC [N][Hs][Ws][C0] (+ [N][Hs][Ws][C1], virtual concat) */
  int32_t Ho, Wo, K;         /* output bf16 NHWC [N][Ho][Wo][K] */
  int32_t mode;              /* 0: 3x3 stride 1 pad 1; 1: 3x3 stride 2 pad 1; 2: nearest-x2 gather, 3x3 s1 p1;
                                3: 1x1 (the centre tap of a 3x3 on 1x1 images) */
  const void* src0;
  const void* src1;
  const void* wgt;           /* bf16 [K][T][C0 + C1], T = 9 (modes 0-2) or 1: fmd_prep_weights mode 0 */
  const float* st0;          /* GroupNorm prologue when non-NULL: statistics slab of src0 [N*Hs*Ws/rows0][C0][2] */
  int32_t rows0;             /*   (sum, sum of squares per rows0-pixel block of one image) */
  const float* st1;          /* ... of src1 (C1 > 0) */
  int32_t rows1;
  int32_t G;                 /* groups */
  float eps;
  const float* gamma;        /* [C0 + C1] or NULL */
  const float* beta;
  const float* emb;          /* scale-shift norm: [N][emb_stride] scale | shift, or NULL */
  int32_t emb_stride;
  int32_t silu;              /* SiLU after the affine */
  const void* src2;          /* 1x1 segment (ResBlock skip conv) over raw (src2 | src3) at the OUTPUT pixels, */
  const void* src3;          /*   bf16 [N][Ho][Wo][C2] (+ [N][Ho][Wo][C3]); C2 = 0: none (modes 0 and 3 only) */
  int32_t C2, C3;
  const void* wgt2;          /* bf16 [K][C2 + C3] */
  const float* bias;         /* [K] or NULL */
  const float* bias2;        /* [K] or NULL (skip-conv bias) */
  const float* bias_nc;      /* per-sample bias [N][bias_nc_stride] (time-embedding add) or NULL */
  int32_t bias_nc_stride;    /* 0: K */
  const void* resid;         /* bf16 [N][Ho][Wo][K] or NULL */
  void* out;
  float* stats;              /* NULL or [N*Ho*Wo/srows][K][2] of the bf16 outputs, srows = 64 if Ho*Wo % 64 == 0
                                else Ho*Wo (one row per image) */
  float* part;               /* split of the reduction over input channels (grids smaller than the chip): fp32
                                partial tiles, part_bytes bytes; NULL: no split */
  int64_t part_bytes;
  uint32_t* tickets;         /* [n_tickets] arrival counters of the in-launch combine: zero before first use, left
                                zero by every completed launch; one set per stream (launches on it serialise) */
  int32_t n_tickets;
  int32_t split;             /* parts: 0 chosen by the plan (enough workgroups for the chip), 1 none, 2..16 forced */
} fmd_conv_small_desc;
/* LDS bytes the launch needs (> 0), or a negative code when the problem does not qualify (geometry, channel
 * counts, or more than one CU's LDS). */
int fmd_conv_small_plan(const fmd_conv_small_desc* d);
/* The number of parts the plan splits the reduction into (>= 1), or the plan's negative code. */
int fmd_conv_small_split(const fmd_conv_small_desc* d);
int fmd_conv_small(const fmd_conv_small_desc* d, fmd_stream_t s);

/* UNet output head: out = conv3x3(SiLU(a*h + b)) to K <= 8 channels, fp32 NHWC [N][H][W][8]
 * (channels >= K zero), replacing the final GroupNorm -> SiLU -> ConvND of
 * src/models/unet/unet.py:286-293 (unet_diffusers_nd.py conv_norm_out/conv_act/conv_out).
 * D == 0: 2-D, h bf16 NHWC [N][H][W][C], w fp32 [K][C][3][3] (reference layout).
 * D >= 1: 3-D (ConvND with dims=3), h [N][D][H][W][C], w [K][C][3][3][3], out [N][D][H][W][8], zero depth
 * padding; K <= 2.  pro_a/pro_b: [N][C] GroupNorm affine; H, W multiples of 16, C a multiple of 32. */
int fmd_head_fwd(const void* h, int32_t N, int32_t D, int32_t H, int32_t W, int32_t C, const float* pro_a,
                 const float* pro_b, const float* w, const float* bias, int32_t K, float* out, fmd_stream_t s);
/* Data gradient of the head: dz = silu'(a*h + b) * conv^T(dpred) (bf16, h's layout) and the
 * GroupNorm-backward sums (sum dz, sum dz*h) per 64-pixel slab row: stats [N*D*H*W/64][C][2].
 * dpred: bf16 [..][8] in h's layout; D as in fmd_head_fwd. */
int fmd_head_dgrad(const void* dpred, const float* w, int32_t K, const void* h, const float* pro_a, const float* pro_b,
                   int32_t N, int32_t D, int32_t H, int32_t W, int32_t C, void* dz, float* stats, fmd_stream_t s);
/* Weight gradient of the head: dw[K][C][taps] += sum_p dpred (x) SiLU(a*h + b), db[K] += sum_p dpred. */
int64_t fmd_head_wgrad_workspace(int32_t N, int32_t D, int32_t H, int32_t W, int32_t C, int32_t K);
int fmd_head_wgrad(const void* dpred, int32_t K, const void* h, const float* pro_a, const float* pro_b, int32_t N,
                   int32_t D, int32_t H, int32_t W, int32_t C, float* dw, float* db, float* ws, fmd_stream_t s);

/* Weight-gradient GEMM: dW[K][C][kh][kw] (+)= sum_p dY[p][K] x gather(src)[p][tap][C]
 * with the same gather/prologue as the forward; db[K] (+)= sum_p dY[p][K].
 * Replaces autograd of nn.Conv2d weight/bias (convolution.py:53). */
typedef struct fmd_wgrad_desc {
  int32_t N, Hs, Ws, C0, C1, Ho, Wo, K, ks, stride, pad, upsample;
  const void* src0; const void* src1;
  const float* pro_a; const float* pro_b; int32_t pro_silu;
  const void* dy;           /* bf16 [N][Ho][Wo][ldy], first K channels used */
  int32_t ldy;              /* dy row stride in elements (0 -> K) */
  float* dw;                /* fp32 [K][C][ks][ks] (reference layout) */
  float* db;                /* fp32 [K] or NULL */
  int32_t accumulate;
  float* ws;                /* fp32 workspace, size fmd_wgrad_workspace() floats */
  int32_t splits;           /* split-K over pixels (halo path: over 8x16-pixel tiles) */
  int32_t force_generic;    /* 1: never use the halo-tiled kernel (tests) */
  int32_t Ds, Do;           /* 3-D: stored / output depth (0 = 2-D); dw [K][C][ks][ks][ks] */
} fmd_wgrad_desc;

/* Dispatches 3x3 stride-1 problems (K % 128 == 0, C % 64 == 0, Ho % 8 == 0, Wo % 16 == 0) to the
 * halo-tiled kernel (csrc/wgrad_halo.hip), everything else to the per-tap kernel (csrc/wgrad.hip). */
int fmd_wgrad(const fmd_wgrad_desc* d, fmd_stream_t s);
/* Halo-tiled 3x3 weight gradient (partial slabs only, no reduce); returns 1 when not applicable. */
int fmd_wgrad_halo(const fmd_wgrad_desc* d, fmd_stream_t s);
int64_t fmd_wgrad_workspace(const fmd_wgrad_desc* d);

/* ------------------------------------------------------------- groupnorm
 * nn.GroupNorm (src/nn/ops/normalization.py:11-19, attention.py:97) is never
 * materialised: producers emit per-channel sums, fmd_gn_prep folds mean/rstd,
 * gamma/beta and the ResBlock scale/shift into a per-(n,c) affine consumed by
 * the conv prologue. */
int fmd_channel_stats(const void* x, const void* y0, const void* y1, int32_t C0, int32_t N, int32_t HW, int32_t C,
                      int32_t rows, float* out /* [N*HW/rows][C][2] */, fmd_stream_t s);
/* Slab fold: out[j] = sum of slab rows [j*fold, (j+1)*fold) of a [rows_total][C][2] statistics slab (fold must not
 * straddle images: (HW/rows) % fold == 0).  Used before fmd_gn_prep / fmd_gn_bwd_prep on slabs with thousands of
 * rows per image (config E's 128^3 levels). */
int fmd_stats_fold(const float* slab, int64_t rows_total, int32_t C, int32_t fold, float* out, fmd_stream_t s);
int fmd_gn_prep(const float* st0, int32_t rows0, const float* st1, int32_t rows1, int32_t N, int32_t HW,
                int32_t C0, int32_t C1, int32_t G, float eps, const float* gamma, const float* beta,
                const float* emb, int32_t emb_stride, int32_t emb_mode /*0 none,1 scale-shift*/,
                float* a, float* b, float* mean_rstd, fmd_stream_t s);
/* emb_mode 0: plain GN; 1: scale/shift (demb = [dscale | dshift]); 2: embedding added to the GN
 * input (demb[n][c] = sum_hw dx, from the forward channel sums fwd_st of x). */
int fmd_gn_bwd_prep(const float* s12, int32_t rows, int32_t N, int32_t HW, int32_t C, int32_t G,
                    const float* mean_rstd, const float* gamma, const float* beta, const float* emb,
                    int32_t emb_stride, int32_t emb_mode, float* P, float* Q, float* R,
                    float* dgamma, float* dbeta, float* demb, int32_t demb_stride, const float* fwd_st,
                    int32_t fwd_rows, float* ws /* [N][C][2] scratch */, fmd_stream_t s);
/* Deferred gamma/beta gradients: fmd_gn_bwd_prep called with dgamma = dbeta = NULL leaves the per-(n,c)
 * partials in its ws; one fmd_gn_gb_fold launch (<= FMD_GB_MAX jobs) then adds sum_n of every job's
 * partials to its dgamma/dbeta -- one launch per backward pass instead of one per GroupNorm. */
#define FMD_GB_MAX 64
typedef struct {
  const float* ws;   /* [N][C][2] (dgamma, dbeta) partials */
  float* dgamma;     /* [C] += , may be NULL */
  float* dbeta;      /* [C] += , may be NULL */
  int32_t N, C;
} fmd_gb_job;
int fmd_gn_gb_fold(const fmd_gb_job* jobs, int32_t njobs, fmd_stream_t s);
/* t = SiLU(a*x + b) (silu != 0) or a*x + b over the concat x0|x1 (bf16 [M][C0+C1]): the GroupNorm
 * prologue materialised once for its consumers. */
/* Whole GroupNorm forward of a small level (HW * C/G <= 16384) in one launch, straight from x0|x1: per
 * (n, group) statistics, a/b (+ emb scale/shift, emb_mode 1), mean/rstd, and t = [SiLU](a*x + b) over the
 * channel concat (= fmd_channel_stats + fmd_gn_prep + fmd_gn_apply_fwd).  C/G % 4 == 0, C0 % 4 == 0. */
int fmd_gn_fused_apply(const void* x0, const void* x1, int32_t C0, int32_t C1, int32_t N, int32_t HW, int32_t G,
                       float eps, const float* gamma, const float* beta, const float* emb, int32_t emb_stride,
                       int32_t emb_mode, int32_t silu, float* a, float* b, float* mean_rstd, void* t,
                       fmd_stream_t s);
int fmd_gn_apply_fwd(const void* x0, const void* x1, int32_t C0, int32_t C1, int64_t M, int32_t HW,
                     const float* a, const float* b, int32_t silu, void* t, fmd_stream_t s);

/* ResBlockND dropout (replaces nn.Dropout in out_layers, src/nn/blocks/residual.py:117): y = x * keep / (1-p)
 * over NHWC bf16 [M pixels][C], keep = hash(seed[0], salt, element index) >= p * 2^32 (regenerated, not
 * stored).  With ep_x (bf16 [M][C]) and ep_a/ep_b ([N][C] fp32, N = M / HW) it is the backward through the
 * dropout and the GN+SiLU prologue: y = x * keep / (1-p) * silu'(ep_a * ep_x + ep_b).  x == y is allowed. */
int fmd_dropout_apply(const void* x, int32_t C, int64_t M, int32_t HW, float p, const int32_t* seed, uint32_t salt,
                      const void* ep_x, const float* ep_a, const float* ep_b, void* y, fmd_stream_t s);
int fmd_gn_bwd_apply(const void* dz, const void* x0, const void* x1, int32_t C0, int32_t C1, int64_t M,
                     int32_t HW, const float* P, const float* Q, const float* R, const void* extra,
                     void* dx0, int32_t acc0, void* dx1, int32_t acc1, fmd_stream_t s);

/* -------------------------------------------------- weights and layouts
 * fp32 reference-layout conv weight -> bf16 kernel layout.  mode 0: [Kpad][T][Cpad]
 * forward; mode 1: [Cpad][T][Kpad] data gradient (transposed gather); mode 2:
 * [Cpad][16][Kpad] data gradient of nearest-x2 upsample + 3x3 conv (4x4 taps). */
int fmd_prep_weights(const float* w, int32_t K, int32_t C, int32_t ks, int32_t mode, int32_t Kpad, int32_t Cpad,
                     void* out, fmd_stream_t s);
/* Same for any tap count T (w [K][C][T], e.g. T = 27 for a 3x3x3 kernel); modes 0, 1 and 3 (3 = mode 1
 * with the taps reversed: the stride-1 data gradient as a forward gather). */
int fmd_prep_weights_t(const float* w, int32_t K, int32_t C, int32_t T, int32_t mode, int32_t Kpad, int32_t Cpad,
                       void* out, fmd_stream_t s);
/* All bf16 weight layouts of a model in one launch (after each optimizer step).  jobs: device int64
 * [njobs][16], one per fp32 master w[K][C][ks*ks] = {w, K | C<<32, ks | nout<<32, first block | ktiles<<32,
 * then nout (<= 6) pairs {out, mode | kind<<8 | R<<16 | Cc<<40}}; kind 0 = the fmd_prep_weights layout
 * (R rows x T x Cc), kind 1 = its halo tiles.  A block covers a 32x32 (k, c) tile of one master; jobs
 * sorted by first block; nblocks = total. */
int fmd_prep_weights_batch(const void* jobs, int32_t njobs, int32_t nblocks, fmd_stream_t s);
/* The same for cubic 3x3x3 masters w[K][C][27] (job ks = 3): blocks cover 16 (k) x 32 (c) tiles (ktiles counts
 * 16-row k tiles); kinds 0 / 1 as above with T = 27, and kind 2 = the depth-tap halo kernel's tiles of the
 * [R][3*Cr][3][3] view (channel block kz*Cr + c = depth tap kz of channel c; Cr = Cc rounded up to 32):
 * [ceil(R/128)][3*Cr/32][9][4][128][8] (modes 0 and 3). */
int fmd_prep_weights_batch_cubic(const void* jobs, int32_t njobs, int32_t nblocks, fmd_stream_t s);
int fmd_nchw_to_nhwc(const float* x, int32_t N, int32_t C, int32_t HW, int32_t Cpad, void* y, fmd_stream_t s);
int fmd_nhwc_to_nchw(const void* y, int32_t src_f32, int32_t N, int32_t C, int32_t HW, int32_t Cs, float* x,
                     fmd_stream_t s);
/* Parameter-free resampling by 2 along the dims whose factor (fz, fy, fx) is 2, NDHWC bf16 (2-D: D = 1; 1-D:
 * D = H = 1).  up = 0: dst[low] (+)= scale * sum of src's 2^d block -- AvgPoolND(kernel=stride=2)
 * (src/nn/ops/pooling.py:33-53, scale 1/2^d; DownsampleND(use_conv=False), upsampling.py:52-58) and the
 * nearest-x2 data gradient (scale 1).  up = 1: dst[high] (+)= scale * src[high >> 1] -- UpsampleND(use_conv=
 * False)'s F.interpolate(scale_factor=2, mode="nearest") (upsampling.py:24-29, scale 1) and the avg-pool data
 * gradient (scale 1/2^d).  High extents are 2*low or 2*low + 1 (floor pooling of an odd extent). */
int fmd_resample2(const void* src, int32_t N, int32_t Dl, int32_t Hl, int32_t Wl, int32_t Dh, int32_t Hh, int32_t Wh,
                  int32_t C, int32_t fz, int32_t fy, int32_t fx, int32_t up, float scale, void* dst, int32_t acc,
                  fmd_stream_t s);
int fmd_sum_pool2(const void* src, int32_t N, int32_t H, int32_t W, int32_t C, void* dst, int32_t acc, fmd_stream_t s);
/* dst[n][z][y][x][c] (+)= sum of the 2x2x2 block of src (bf16 NDHWC, src 2D x 2H x 2W): the data gradient
 * of a nearest-x2 3-D upsample. */
int fmd_sum_pool2_3d(const void* src, int32_t N, int32_t D, int32_t H, int32_t W, int32_t C, void* dst,
                     int32_t acc, fmd_stream_t s);
int fmd_add_bf16(const void* a, void* dst, int64_t n, fmd_stream_t s);

/* ------------------------------------------------------ time embedding
 * timestep_embedding (src/nn/ops/time_embedding.py:4-32), the time MLP
 * (src/models/unet/unet.py:117-121, src/models/unet/utils.py:9-24) and the
 * ResBlock emb_layers (src/nn/blocks/residual.py:63-68,102-104). */
/* t_eff = t*t_scale, truncated to an integer when t_trunc (the FM trainer's (t*(N-1)).long()) */
int fmd_timestep_embedding(const float* t, int32_t N, int32_t dim, int32_t flip, int32_t shift, float max_period,
                           float t_scale, int32_t t_trunc, float* out, fmd_stream_t s);
int fmd_linear(const float* x, int32_t B, int32_t I, const float* w, const float* b, int32_t O, int32_t in_silu,
               float* y, int32_t y_stride, fmd_stream_t s);
int fmd_linear_bwd(const float* x, int32_t B, int32_t I, const float* w, int32_t O, int32_t in_silu,
                   const float* dy, int32_t dy_stride, float* dx, int32_t dx_acc, float* dw, float* db,
                   fmd_stream_t s);
/* Grouped linears: every ResBlock emb_layers projection of the UNet in one launch.  groups: device
 * array of {const float* w; const float* b; float* dw; float* db; int64 O; int64 off} (row offset of the
 * group in y / dy); blocks: device int2 array {group, first row} of 64-row blocks.  The backward
 * accumulates dW/db (+=) and writes / accumulates dx (with SiLU' when in_silu). */
int fmd_grouped_linear(const float* x, int32_t B, int32_t I, const void* groups, const void* blocks, int32_t nblk,
                       int32_t in_silu, float* y, int32_t y_stride, fmd_stream_t s);
int64_t fmd_grouped_linear_bwd_workspace(int32_t B, int32_t I, int32_t nblk);
int fmd_grouped_linear_bwd(const float* x, int32_t B, int32_t I, const void* groups, const void* blocks,
                           int32_t nblk, int32_t in_silu, const float* dy, int32_t dy_stride, float* dx,
                           int32_t dx_acc, float* ws, fmd_stream_t s);
int fmd_silu_bwd_f32(const float* x, const float* dy, float* dx, int64_t n, fmd_stream_t s);

/* ----------------------------------------------------------- attention
 * Softmax attention (F.scaled_dot_product_attention inside SpatialSelfAttention / DiffusersAttentionND /
 * SpatialCrossAttention) runs on the MFMA kernels declared further down (fmd_attn_pack / fmd_attn_mfma_fwd /
 * fmd_attn_mfma_bwd / fmd_attn_unpack). */
/* LinearQKVAttention (src/nn/blocks/attention.py:53-70) inside SpatialSelfAttention(use_linear=True)
 * (attention.py:104-117; same raw head split): out = softmax_d(q) (softmax_tokens(k)^T v / (sum ks + eps)).
 * ``state`` (fmd_linear_attention_state floats) is written by the forward and read by the backward;
 * ``ws`` holds fmd_linear_attention_workspace floats. dh <= 64. */
/* SpatialCrossAttention (attention.py:120-189): q [B][Tq][inner] (q_proj output), kv [B][Tk][2*inner]
 * (kv_proj output), raw head split q.reshape(b, heads, Tq, dh), kv.reshape(b, heads, Tk, 2dh).chunk(2).
 * linear must be 1: LinearQKVAttention (lse_or_state = fmd_linear_attention_state floats, ws = workspace);
 * linear = 0 returns -2 (softmax cross-attention is fmd_attn_mfma_fwd / fmd_attn_mfma_bwd). */
int fmd_cross_attention_fwd(const void* q, const void* kv, int32_t B, int32_t Tq, int32_t Tk, int32_t heads,
                            int32_t dh, int32_t raw, int32_t linear, float eps, void* o, float* lse_or_state,
                            float* ws, fmd_stream_t s);
int fmd_cross_attention_bwd(const void* q, const void* kv, const void* o, const void* dout, const float* lse_or_state,
                            float* ws_or_delta, int32_t B, int32_t Tq, int32_t Tk, int32_t heads, int32_t dh,
                            int32_t raw, int32_t linear, float eps, void* dq, void* dkv, fmd_stream_t s);
/* Softmax attention on MFMA (csrc/attention_mfma.hip), the path behind every softmax attention block
 * (attention.py:42-44, 115, 185, 269).  The reference's head split (raw reshape or view/transpose; self:
 * src_q = src_kv = qkv [B][T][3*inner]; cross: src_q = q [B][Tq][inner], src_kv = kv [B][Tk][2*inner];
 * which 3 = the attention output o [B][Tq][inner]) is undone into canonical bf16 planes
 * [B*heads][rows][fmd_attn_head_pad(dh)] (q/o/dq plane cq, k plane ck, v plane cv; pad zero-filled).
 * fmd_attn_pack gathers planes which0..which1 (0 q, 1 k, 2 v, 3 o/dout into cq); fmd_attn_unpack scatters
 * them back (0..2 into dst_q for self attention = dqkv, into dst_q / dst_kv for cross; 3 into dst_q).
 * fmd_attn_mfma_fwd: co = softmax(cq ck^T / sqrt(dh)) cv, lse [B*heads][Tq] (natural log).
 * fmd_attn_mfma_bwd: delta [B*heads][Tq] scratch, writes cdq, cdk, cdv.  dh <= 64. */
int32_t fmd_attn_head_pad(int32_t dh);
int fmd_attn_pack(const void* src_q, const void* src_kv, int32_t B, int32_t Tq, int32_t Tk, int32_t heads,
                  int32_t dh, int32_t raw, int32_t cross, int32_t which0, int32_t which1, void* cq, void* ck,
                  void* cv, fmd_stream_t s);
int fmd_attn_unpack(const void* cq, const void* ck, const void* cv, int32_t B, int32_t Tq, int32_t Tk,
                    int32_t heads, int32_t dh, int32_t raw, int32_t cross, int32_t which0, int32_t which1,
                    void* dst_q, void* dst_kv, fmd_stream_t s);
int fmd_attn_mfma_fwd(const void* cq, const void* ck, const void* cv, int32_t BH, int32_t Tq, int32_t Tk,
                      int32_t dh, void* co, float* lse, fmd_stream_t s);
int fmd_attn_mfma_bwd(const void* cq, const void* ck, const void* cv, const void* co, const void* cdo,
                      const float* lse, float* delta, int32_t BH, int32_t Tq, int32_t Tk, int32_t dh, void* cdq,
                      void* cdk, void* cdv, fmd_stream_t s);
/* context_norm of SpatialCrossAttention: GroupNorm over the fp32 context ((N, C, T) or token-major (N, T, C))
 * -> bf16 [N][T][Cpad] (zero pad channels); mr [N][groups][2] = mean, rstd.  The backward accumulates
 * dgamma / dbeta only (the context is conditioning data). */
int fmd_context_norm_fwd(const float* ctx, int32_t N, int32_t C, int32_t T, int32_t tok_major, int32_t groups,
                         float eps, const float* gamma, const float* beta, int32_t Cpad, void* out, float* mr,
                         fmd_stream_t s);
int fmd_context_norm_bwd(const float* ctx, int32_t N, int32_t C, int32_t T, int32_t tok_major, int32_t groups,
                         const float* mr, const void* dout, int32_t Cpad, float* dgamma, float* dbeta,
                         fmd_stream_t s);
size_t fmd_linear_attention_workspace(int32_t B, int32_t heads);
size_t fmd_linear_attention_state(int32_t B, int32_t heads);
int fmd_linear_attention_fwd(const void* qkv, int32_t B, int32_t T, int32_t heads, int32_t dh, int32_t raw,
                             float eps, void* o, float* state, float* ws, fmd_stream_t s);
int fmd_linear_attention_bwd(const void* qkv, const void* dout, const float* state, float* ws, int32_t B, int32_t T,
                             int32_t heads, int32_t dh, int32_t raw, float eps, void* dqkv, fmd_stream_t s);

/* ------------------------------------------ train step / sampler / optim
 * FM input x_t = (1-t)x0 + t*eps and DDPM add_noise (flow_matching_lib.py:151-158,
 * diffusion_lib.py:154-160) -> NHWC model input with the concatenated
 * conditioning; MSE loss + gradient (flow_matching_lib.py:166-167); the
 * FlowMatchEuler / DDPM step (diffusers, called at src/pipelines/utils.py:218);
 * torch.optim.AdamW (flow_matching_lib.py:73,177). */
/* x channels: ca&&cb: ca[n]*x0 + cb[n]*noise (DDPM add_noise); ca only: (1-ca[n])*x0 + ca[n]*noise
 * (FM, ca = t); neither: noise (sampler input). */
int fmd_noise_prepare(const float* x0, const float* noise, const float* ca, const float* cb, const float* cond,
                      int32_t N, int32_t HW, int32_t Cx, int32_t Cc, int32_t Cpad, void* inp, fmd_stream_t s);
/* diffusers DDPMScheduler.add_noise (diffusion_lib.py:158, diffusion_utils.py:162/222) in fp32:
 * out[n] = sqrt_acp[t[n]] * x0[n] + sqrt_1m_acp[t[n]] * noise[n] over per_sample elements per sample,
 * torch's operation order (two rounded products, one rounded add): bit-exact with the eager op.
 * sqrt_acp / sqrt_1m_acp: [num_train_timesteps] fp32 tables; timesteps: int64 [N] on the device. */
int fmd_add_noise(const float* x0, const float* noise, const float* sqrt_acp, const float* sqrt_1m_acp,
                  const int64_t* timesteps, int32_t N, int64_t per_sample, float* out, fmd_stream_t s);
int fmd_mse(const float* pred, int32_t Kpad, const float* ta, const float* tb, float tb_sign, int32_t N, int32_t Cx,
            int32_t HW, float grad_scale, float* partial, int32_t max_blocks, float* loss, void* dpred,
            fmd_stream_t s);
int fmd_adamw(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2, float eps,
              float wd, float bc1, float bc2, fmd_stream_t s);
/* AdamW with the step count on device and get_cosine_schedule_with_warmup's LR computed in-kernel
 * (graph-replayable train step); g is scaled by grad_scale first. */
int fmd_adamw_sched(float* p, const float* g, float* m, float* v, int64_t n, const int32_t* step_ctr, float base_lr,
                    int32_t warmup, int32_t total, float beta1, float beta2, float eps, float wd, float grad_scale,
                    fmd_stream_t s);
int fmd_flow_euler(float* x, const float* v, int32_t Kpad, const float* sigmas, const int32_t* index, int32_t N,
                   int32_t Cx, int32_t HW, const float* cond, int32_t Cc, int32_t Cpad, void* next, fmd_stream_t s);
/* noise: DDPM variance noise, a per-step table whose row 0 belongs to step noise_base (row = index - noise_base),
 * or, with noise_base < 0, one [N][Cx][HW] buffer refilled before every step; NULL for DDIM / the last step. */
int fmd_ddpm_step(float* x, const float* eps, int32_t Kpad, const float* coef, const int32_t* index,
                  const float* noise, int32_t noise_base, int32_t N, int32_t Cx, int32_t HW, const float* cond,
                  int32_t Cc, int32_t Cpad, void* next, fmd_stream_t s);
int fmd_fill_from_table(const float* table, const int32_t* index, float* out, int32_t N, fmd_stream_t s);
/* out = sum_k c[k] * in[k] over n fp32 elements: the multistep scheduler updates (DPM-Solver / UniPC,
 * replaces diffusers' DPMSolverMultistepScheduler.step / UniPCMultistepScheduler.step tensor arithmetic,
 * called at src/pipelines/utils.py:218).  out may alias an input.  n % 4 == 0 needs 16-byte alignment. */
#define FMD_LINCOMB_MAX 6
typedef struct {
  float* out;
  const float* in[FMD_LINCOMB_MAX];
  float c[FMD_LINCOMB_MAX];
  int32_t nin;
  int64_t n;
} fmd_lincomb_desc;
int fmd_lincomb(const fmd_lincomb_desc* d, fmd_stream_t s);
/* One multistep-solver step with every scalar taken from row index[0] of a per-step coefficient table, so a
 * whole DPM-Solver / UniPC sampling loop replays from one captured step (the graph-replayed form of the
 * DPMSolverMultistepScheduler.step / UniPCMultistepScheduler.step arithmetic, reference call site
 * src/pipelines/utils.py:218).  Per element of the sample (step i = index[0], r(j) = ring[j & 3]):
 *   m      = c[0]*x + c[1]*eps                                   (data prediction; dpmsolver: eps itself)
 *   r(i)   = m
 *   xc     = c[2] != 0 ? c[3]*last + c[4]*r(i-1) + c[5]*r(i-2) + c[6]*r(i-3) + c[7]*m : x   (UniPC corrector)
 *   last   = xc                                                  (if last != NULL)
 *   x      = c[8]*xc + c[9]*r(i) + c[10]*r(i-1) + c[11]*r(i-2)   (predictor / solver update)
 * each sum accumulated left to right from 0 with fused multiply-adds, as fmd_lincomb does, so the step equals
 * the eager scheduler's fmd_lincomb calls on the same coefficients.  x: [N][Cx][HW] fp32; eps: the UNet
 * output [N*HW][Kpad] fp32; ring / last: [N][Cx][HW] fp32; next (optional): the next model input
 * (NHWC bf16 [N*HW][Cpad], x then cond channels, zero padded) as fmd_flow_euler writes it. */
#define FMD_SCHED_NCOEF 12
typedef struct {
  float* x;
  const float* eps;
  float* ring[4];
  float* last;
  const float* coef;        /* [steps][FMD_SCHED_NCOEF] */
  const int32_t* index;
  int32_t N, Cx, HW, Kpad;
  const float* cond;
  int32_t Cc, Cpad;
  void* next;
} fmd_sched_step_desc;
int fmd_sched_step(const fmd_sched_step_desc* d, fmd_stream_t s);
/* out[0:n] = table[index[0]*n : (index[0]+1)*n] -- a per-step row (e.g. precomputed time embeddings of a
 * sampling schedule) selected by a device-side step counter, so the step stays graph-replayable. */
int fmd_gather_row(const float* table, const int32_t* index, int64_t n, float* out, fmd_stream_t s);
int fmd_counter_add(int32_t* c, int32_t v, fmd_stream_t s);
/* y = x (NHWC bf16, Cpad channels per pixel) with channels [0, C) mapped to scale * x + shift: the model
 * input centring of UNetDiffusersND(center_input_sample=True), `x = 2 * x - 1.0`
 * (src/models/unet/unet_diffusers_nd.py:156-157), applied to the packed input (one extra bf16 rounding). */
int fmd_affine_channels(const void* x, int32_t C, int32_t Cpad, int64_t npix, float scale, float shift, void* y,
                        fmd_stream_t s);

#ifdef __cplusplus
}
#endif
#endif
