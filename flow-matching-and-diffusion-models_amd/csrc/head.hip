// Output head of the UNet: GroupNorm -> SiLU -> 3x3 conv to K <= 8 channels (fp32 output,
// channels padded to Kp = 8), and its backward.  Replaces the reference's final
// ``out = nn.Sequential(norm, SiLU, ConvND(model_channels -> out_channels, 3))``
// (src/models/unet/unet.py:286-293 / unet_diffusers_nd.py conv_norm_out + conv_out) and the
// autograd of that conv (src/nn/ops/convolution.py:53).
//
// K is 1 for every BASELINE config: an MFMA tile would waste 15/16 of its rows and the
// per-tap implicit GEMM re-applies the GN/SiLU transform 9 times per element, so these are
// VALU kernels around a once-per-element transform:
//   head_fwd   : 16x16-pixel tile per workgroup, thread = pixel; per 32-channel chunk the
//                transformed (18x18) halo is staged once in LDS (chunk-major planes, as in
//                conv_halo.hip) and every tap reads it; weights of the chunk in LDS as bf16 pairs
//                (broadcast); taps are v_dot2c_f32_bf16 on the packed halo (fp32 accumulate).
//   head_dgrad : thread = 8 channels x one tile row; dpred's 18x18 halo (Kp = 8 bf16 = 16 B per
//                pixel) in LDS; epilogue = SiLU' of the forward pre-activation, bf16 store and the
//                GroupNorm-backward sums (sum dz, sum dz*x) per 64-pixel slab row.
//   head_wgrad : per chunk, thread = (8-channel group, tap, pixel phase) summing dpred * t over
//                the tile from LDS; per-workgroup partials [wg][K][C][9] + [wg][K] reduced by
//                slot_sum + head_wgrad_finish into the reference [K][C][3][3] layout.
#include "common.h"
#include "../../include/fmdiff.h"

namespace {

constexpr int HT = 16;                 // tile edge
constexpr int HR = HT + 2;             // halo row (18)
constexpr int HPOS = HR * HR;          // 324
constexpr int HPADP = 336;             // plane stride (16-byte rows), == 0 mod 16
constexpr int CK = 32;                 // channels per chunk
constexpr int KCP = CK / 8;            // 16-byte planes per chunk
constexpr int NTH = 256;

FMD_DEV int hp_pos(int h) { return (h >> 5) * 8 + (h & 7); }
FMD_DEV int hp_kc(int h) { return (h >> 3) & (KCP - 1); }

// stage the GN+SiLU-transformed halo of channels [c0, c0+32) of tile (ty0, tx0) of slice sl (= n*D + z;
// sample n's GroupNorm affine) into halo[4][336].  A thread's pieces q = tid + 256 i share one 8-channel group
// (hp_kc), so its affine is loaded once, and all its halo loads are issued before the first transform: one memory
// latency per chunk instead of one per piece (the loop form was a chain of ~5 dependent round trips per chunk:
// head_fwd 72 -> 60 us on the 8x256^2 head; a further register prefetch of the next chunk's halo measured no gain)
FMD_DEV void stage_halo(u32x4* halo, const bf16r* __restrict__ h, int sl, int n, int H, int W, int C, int ty0,
                        int tx0, int c0, const float* __restrict__ pa, const float* __restrict__ pb, int tid) {
  constexpr int TOT = ((HPOS + 7) / 8) * 8 * KCP;   // 1312 pieces
  constexpr int NP = (TOT + NTH - 1) / NTH;         // pieces per thread (6)
  const int kc = hp_kc(tid);
  const int c = c0 + kc * 8;
  const f32x4 a0 = *(const f32x4*)(pa + (size_t)n * C + c), a1 = *(const f32x4*)(pa + (size_t)n * C + c + 4);
  const f32x4 b0 = *(const f32x4*)(pb + (size_t)n * C + c), b1 = *(const f32x4*)(pb + (size_t)n * C + c + 4);
  u32x4 r[NP];
  bool ok[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int q = tid + NTH * i, pos = hp_pos(q);
    const int y = ty0 - 1 + pos / HR, x = tx0 - 1 + pos % HR;
    ok[i] = q < TOT && pos < HPOS && y >= 0 && y < H && x >= 0 && x < W;
    r[i] = *(const u32x4*)(h + (ok[i] ? ((size_t)(sl * H + y) * W + x) * C + c : (size_t)0));
  }
  const float av[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
  const float bv[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int q = tid + NTH * i, pos = hp_pos(q);
    if (q >= TOT || pos >= HPOS) continue;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (ok[i]) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        v[e] = pack2(siluf_(bf_lo(r[i][e]) * av[2 * e] + bv[2 * e]), siluf_(bf_hi(r[i][e]) * av[2 * e + 1] + bv[2 * e + 1]));
    }
    halo[kc * HPADP + pos] = v;
  }
}

struct HeadArgs {
  const bf16r* h;       // [N][D][H][W][C] GN input (D = 1 for 2-D data)
  const float* pa;      // [N][C]
  const float* pb;
  const float* w;       // [K][C][T] (T = 9: [3][3]; T = 27: [3][3][3])
  const float* bias;    // [K] or null
  const bf16r* dpred;   // [N][H][W][8]
  float* out;           // fp32 [N][H][W][Kp]
  bf16r* dz;            // [N][H][W][C]
  float* stats;         // [N*H*W/64][C][2]
  float* ws;            // wgrad partials
  int N, D, H, W, C, K, Kp, T;
  int tiles_x, tiles_y, ntiles, tiles_per_wg;
};

// tile -> (slice sl = n*D + z, sample n, depth z, tile origin); tiles run x, then y, then slice
struct TilePos {
  int sl, n, z, ty0, tx0;
};
FMD_DEV TilePos tile_pos(const HeadArgs& A, int t) {
  const int per = A.tiles_x * A.tiles_y;
  TilePos P;
  P.sl = t / per;
  const int tr = t - P.sl * per;
  P.n = P.sl / A.D;
  P.z = P.sl - P.n * A.D;
  P.ty0 = (tr / A.tiles_x) * HT;
  P.tx0 = (tr % A.tiles_x) * HT;
  return P;
}

// KZ = 1: 2-D; KZ = 3: 3-D (one depth plane of taps per pass over the chunk, zero depth padding).
// CG chunk groups: a workgroup of CG x 256 threads, group g taking the 32-channel chunks g, g + CG, ... of the tile
// with its own halo / weight buffers, the groups' sums combined in LDS at the end -- for grids of a few tiles (the
// latent UNet's 32^2 head: 32 tiles of 16x16, 4 chunks each; the VAE encoder's 512-channel head: 16 chunks), where a
// single 256-thread group would walk every chunk serially on 32 of the 256 CUs
template <int KT, int KZ, int CG>
__global__ __launch_bounds__(NTH * CG) void head_fwd(const HeadArgs A) {
  __shared__ __attribute__((aligned(16))) u32x4 halo_all[CG][KCP * HPADP];
  __shared__ __attribute__((aligned(16))) unsigned int wl_all[CG][KT][9][CK / 2];   // chunk weights [k][tap][c pair]
  const int tid = threadIdx.x % NTH, grp = threadIdx.x / NTH;
  u32x4* halo = halo_all[grp];
  unsigned int (*wl)[9][CK / 2] = wl_all[grp];
  const TilePos P = tile_pos(A, blockIdx.x);
  const int n = P.n, ty0 = P.ty0, tx0 = P.tx0;
  const int py = tid >> 4, px = tid & 15;
  // two accumulators per output channel (the 8-channel pieces alternate), fp32 throughout
  float acc[KT][2];
#pragma unroll
  for (int k = 0; k < KT; ++k) acc[k][0] = acc[k][1] = 0.f;
  const int rounds = (A.C / CK + CG - 1) / CG;   // every group passes the same barriers
  for (int rd = 0; rd < rounds; ++rd) {
    const int c0 = (rd * CG + grp) * CK;
    const bool act = c0 < A.C;
    for (int kz = 0; kz < KZ; ++kz) {
      const int zz = P.z + kz - KZ / 2;
      if (zz < 0 || zz >= A.D) continue;   // zero depth padding (uniform over the workgroup)
      if (act) {
        stage_halo(halo, A.h, P.sl + zz - P.z, n, A.H, A.W, A.C, ty0, tx0, c0, A.pa, A.pb, tid);
        for (int i = tid; i < KT * 9 * (CK / 2); i += NTH) {
          const int k = i / (9 * (CK / 2)), r = i - k * 9 * (CK / 2), tap = r / (CK / 2), cp = r - tap * (CK / 2);
          const size_t w0 = ((size_t)k * A.C + c0 + 2 * cp) * (9 * KZ) + kz * 9 + tap;
          wl[k][tap][cp] = k < A.K ? pack2(A.w[w0], A.w[w0 + 9 * KZ]) : 0u;
        }
      }
      __syncthreads();
      // bf16 operands straight from LDS into v_dot2c_f32_bf16 (two products per op, fp32 accumulate):
      // no per-tap unpacking of the halo, a quarter of the fp32-FMA form's VALU ops
      if (act) {
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const int pos = (py + tap / 3) * HR + px + tap % 3;
#pragma unroll
          for (int kc = 0; kc < KCP; ++kc) {
            const u32x4 v = halo[kc * HPADP + pos];
#pragma unroll
            for (int k = 0; k < KT; ++k) {
              const u32x4 w = *(const u32x4*)&wl[k][tap][kc * 4];
              float a = acc[k][kc & 1];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                // copy the vector lanes to scalars first: __builtin_bit_cast of an ext_vector element lvalue
                // reads lane 0 (hipcc 7.2), which silently dotted the first channel pair four times
                const unsigned int ve = v[e], we = w[e];
                a = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_, ve), __builtin_bit_cast(bf16x2_, we),
                                                    a, false);
              }
              acc[k][kc & 1] = a;
            }
          }
        }
      }
      __syncthreads();
    }
  }
  float sum[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k) sum[k] = acc[k][0] + acc[k][1];
  if (CG > 1) {   // groups 1.. hand their sums to group 0 through LDS (the halo buffers are free after the barrier)
    float* red = (float*)&halo_all[0][0];
    if (grp > 0) {
#pragma unroll
      for (int k = 0; k < KT; ++k) red[((grp - 1) * KT + k) * NTH + tid] = sum[k];
    }
    __syncthreads();
    if (grp > 0) return;
#pragma unroll
    for (int g = 1; g < CG; ++g)
#pragma unroll
      for (int k = 0; k < KT; ++k) sum[k] += red[((g - 1) * KT + k) * NTH + tid];
  }
  const size_t p = ((size_t)(P.sl * A.H) + ty0 + py) * A.W + tx0 + px;
  float* o = A.out + p * A.Kp;
  for (int k = 0; k < A.Kp; k += 4) {
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int kk = k + e;
      float r = 0.f;
#pragma unroll
      for (int j = 0; j < KT; ++j)
        if (j == kk) r = sum[j];
      v[e] = kk < A.K ? r + (A.bias ? A.bias[kk] : 0.f) : 0.f;
    }
    *(f32x4*)(o + k) = v;
  }
}

// dz[p][c] = silu'(a x + b) * sum_{tap,k} dpred[p - tap + 1][k] W[k][c][tap]; stats (sum dz, sum dz*x).
// KZ = 3 (3-D): the dpred halos of slices z+1, z, z-1 (depth taps 0, 1, 2) and all 27 taps' weights in LDS
template <int KT, int KZ>
__global__ __launch_bounds__(256) void head_dgrad(const HeadArgs A) {
  __shared__ __attribute__((aligned(16))) float dp[KZ][HPOS][KT];          // dpred halos (fp32)
  __shared__ __attribute__((aligned(16))) float wl[9 * KZ][KT][128];       // weights of this 128-channel block
  const int tid = threadIdx.x;
  const TilePos P = tile_pos(A, blockIdx.x);
  const int n = P.n, ty0 = P.ty0, tx0 = P.tx0;
  const int cb0 = blockIdx.y * 128;
  const int g = tid & 15, r = tid >> 4;   // 8 channels x one tile row
  for (int i = tid; i < KZ * HPOS; i += NTH) {
    const int kz = i / HPOS, pos = i - kz * HPOS;
    const int zz = P.z - kz + KZ / 2;
    const int y = ty0 - 1 + pos / HR, x = tx0 - 1 + pos % HR;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (zz >= 0 && zz < A.D && y >= 0 && y < A.H && x >= 0 && x < A.W) {
      const u32x4 q = *(const u32x4*)(A.dpred + ((size_t)((P.sl + zz - P.z) * A.H + y) * A.W + x) * 8);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[2 * e] = bf_lo(q[e]); v[2 * e + 1] = bf_hi(q[e]); }
    }
#pragma unroll
    for (int k = 0; k < KT; ++k) dp[kz][pos][k] = v[k];
  }
  for (int i = tid; i < 9 * KZ * KT * 128; i += NTH) {
    const int tap = i / (KT * 128), rr = i - tap * KT * 128, k = rr / 128, c = rr - k * 128;
    wl[tap][k][c] = (k < A.K && cb0 + c < A.C) ? A.w[((size_t)k * A.C + cb0 + c) * (9 * KZ) + tap] : 0.f;
  }
  __syncthreads();
  const int c = cb0 + g * 8;
  const bool cok = c < A.C;
  float a[8], b[8], s1[8], s2[8];
  if (cok) {
    const f32x4 a0 = *(const f32x4*)(A.pa + (size_t)n * A.C + c), a1 = *(const f32x4*)(A.pa + (size_t)n * A.C + c + 4);
    const f32x4 b0 = *(const f32x4*)(A.pb + (size_t)n * A.C + c), b1 = *(const f32x4*)(A.pb + (size_t)n * A.C + c + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { a[e] = a0[e]; a[4 + e] = a1[e]; b[e] = b0[e]; b[4 + e] = b1[e]; }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  for (int x = 0; x < HT; ++x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9 * KZ; ++tap) {
      const int ky = (tap % 9) / 3, kx = tap % 3;
      const int pos = (r + 2 - ky) * HR + x + 2 - kx;
#pragma unroll
      for (int k = 0; k < KT; ++k) {
        const float d = dp[tap / 9][pos][k];
        const f32x4 w0 = *(const f32x4*)&wl[tap][k][g * 8], w1 = *(const f32x4*)&wl[tap][k][g * 8 + 4];
#pragma unroll
        for (int e = 0; e < 4; ++e) { acc[e] += d * w0[e]; acc[4 + e] += d * w1[e]; }
      }
    }
    if (cok) {
      const size_t p = ((size_t)(P.sl * A.H) + ty0 + r) * A.W + tx0 + x;
      const u32x4 xr = *(const u32x4*)(A.h + p * A.C + c);
      u32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x0 = bf_lo(xr[e]), x1 = bf_hi(xr[e]);
        o[e] = pack2(acc[2 * e] * silu_grad(a[2 * e] * x0 + b[2 * e]),
                     acc[2 * e + 1] * silu_grad(a[2 * e + 1] * x1 + b[2 * e + 1]));
        const float w0 = bf_lo(o[e]), w1 = bf_hi(o[e]);
        s1[2 * e] += w0; s2[2 * e] += w0 * x0;
        s1[2 * e + 1] += w1; s2[2 * e + 1] += w1 * x1;
      }
      *(u32x4*)(A.dz + p * A.C + c) = o;
    }
  }
  // the wave's 4 rows x 16 pixels = one 64-pixel slab row: sum lanes g, g+16, g+32, g+48
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    s1[e] += __shfl_xor(s1[e], 16, 64);
    s1[e] += __shfl_xor(s1[e], 32, 64);
    s2[e] += __shfl_xor(s2[e], 16, 64);
    s2[e] += __shfl_xor(s2[e], 32, 64);
  }
  if ((r & 3) == 0 && cok) {
    const int srow = blockIdx.x * 4 + (r >> 2);
    float* sp = A.stats + ((size_t)srow * A.C + c) * 2;
#pragma unroll
    for (int e = 0; e < 8; ++e) { sp[2 * e] = s1[e]; sp[2 * e + 1] = s2[e]; }
  }
}

// per-workgroup partials: slot[wg] = {[k][c][tap] (reference layout per k), [k] bias}; the workgroup
// owns tiles [wg*tpw, (wg+1)*tpw) and keeps its sums in registers across them, chunk by chunk (3-D: and
// depth tap by depth tap, the halo taken from slice z + kz - 1; the bias sums ride on the centre pass)
template <int KT, int KZ>
__global__ __launch_bounds__(256) void head_wgrad(const HeadArgs A) {
  __shared__ __attribute__((aligned(16))) u32x4 halo[KCP * HPADP];
  __shared__ __attribute__((aligned(16))) float dp[256][KT];
  __shared__ __attribute__((aligned(16))) float red[7][36][KT * 8];
  __shared__ float bsum[4][KT];
  const int tid = threadIdx.x;
  const int combo = tid % 36, phase = tid / 36;   // 7 phases x 36 (kc, tap); threads 252..255 only stage
  const int kc = combo / 9, tap = combo % 9;
  const size_t slot = (size_t)KT * A.C * 9 * KZ + KT;
  float* wsw = A.ws + (size_t)blockIdx.x * slot;
  const int t0 = blockIdx.x * A.tiles_per_wg, t1 = min(A.ntiles, t0 + A.tiles_per_wg);
  float dbs[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k) dbs[k] = 0.f;
  for (int c0 = 0; c0 < A.C; c0 += CK)
  for (int kz = 0; kz < KZ; ++kz) {
    const bool bias_pass = c0 == 0 && kz == KZ / 2;
    float acc[KT][8];
#pragma unroll
    for (int k = 0; k < KT; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[k][e] = 0.f;
    for (int t = t0; t < t1; ++t) {
      const TilePos P = tile_pos(A, t);
      const int ty0 = P.ty0, tx0 = P.tx0;
      const int zz = P.z + kz - KZ / 2;
      if (zz < 0 || zz >= A.D) continue;   // zero depth padding: no contribution (uniform over the workgroup)
      {
        const int py = tid >> 4, px = tid & 15;
        const u32x4 q = *(const u32x4*)(A.dpred + (((size_t)(P.sl * A.H) + ty0 + py) * A.W + tx0 + px) * 8);
        const float v[8] = {bf_lo(q[0]), bf_hi(q[0]), bf_lo(q[1]), bf_hi(q[1]),
                            bf_lo(q[2]), bf_hi(q[2]), bf_lo(q[3]), bf_hi(q[3])};
#pragma unroll
        for (int k = 0; k < KT; ++k) {
          dp[tid][k] = v[k];
          if (bias_pass) dbs[k] += v[k];
        }
      }
      stage_halo(halo, A.h, P.sl + zz - P.z, P.n, A.H, A.W, A.C, ty0, tx0, c0, A.pa, A.pb, tid);
      __syncthreads();
      if (phase < 7) {
        for (int p = phase; p < 256; p += 7) {
          const int pos = ((p >> 4) + tap / 3) * HR + (p & 15) + tap % 3;
          const u32x4 v = halo[kc * HPADP + pos];
          const float tv[8] = {bf_lo(v[0]), bf_hi(v[0]), bf_lo(v[1]), bf_hi(v[1]),
                               bf_lo(v[2]), bf_hi(v[2]), bf_lo(v[3]), bf_hi(v[3])};
#pragma unroll
          for (int k = 0; k < KT; ++k) {
            const float d = dp[p][k];
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[k][e] += d * tv[e];
          }
        }
      }
      __syncthreads();
    }
    if (phase < 7) {
#pragma unroll
      for (int k = 0; k < KT; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e) red[phase][combo][k * 8 + e] = acc[k][e];
    }
    __syncthreads();
    // sum the 7 phases; write this chunk's part of the slot
    for (int i = tid; i < 36 * KT * 8; i += NTH) {
      const int cmb = i / (KT * 8), r = i - cmb * KT * 8, k = r / 8, e = r % 8;
      float sum = 0.f;
#pragma unroll
      for (int ph = 0; ph < 7; ++ph) sum += red[ph][cmb][r];
      wsw[((size_t)k * A.C + c0 + (cmb / 9) * 8 + e) * (9 * KZ) + kz * 9 + cmb % 9] = sum;
    }
    __syncthreads();
  }
  // bias partials: every thread summed its own pixel of each tile
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    const float v = wave_sum(dbs[k]);
    if ((tid & 63) == 0) bsum[tid >> 6][k] = v;
  }
  __syncthreads();
  if (tid < KT) wsw[slot - KT + tid] = bsum[0][tid] + bsum[1][tid] + bsum[2][tid] + bsum[3][tid];
}

// out[s][i] = sum over slots g in split s of in[g][i]  (i < len; slots of stride `stride`)
__global__ void slot_sum(const float* __restrict__ in, int nslots, size_t stride, int len, int per_split,
                         float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= len) return;
  const int g0 = blockIdx.y * per_split, g1 = min(nslots, g0 + per_split);
  float s0 = 0.f, s1 = 0.f;
  int g = g0;
  for (; g + 2 <= g1; g += 2) { s0 += in[(size_t)g * stride + i]; s1 += in[(size_t)(g + 1) * stride + i]; }
  if (g < g1) s0 += in[(size_t)g * stride + i];
  out[(size_t)blockIdx.y * len + i] = s0 + s1;
}

// dw[k][c][tap] += sum_s part[s][k][c][tap];  db[k] += sum_s part[s][KT*C*T + k]  (T = 9 or 27 taps)
__global__ void head_wgrad_finish(const float* __restrict__ part, int ns, int KT, int K, int C, int T,
                                  float* __restrict__ dw, float* __restrict__ db) {
  const int len = KT * C * T + KT;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float s = 0.f;
  if (i < K * C * T) {
    for (int g = 0; g < ns; ++g) s += part[(size_t)g * len + i];
    dw[i] += s;
  } else if (db && i >= KT * C * T && i < KT * C * T + K) {
    for (int g = 0; g < ns; ++g) s += part[(size_t)g * len + i];
    db[i - KT * C * T] += s;
  }
}

int kt_of(int K) { return K <= 1 ? 1 : K <= 2 ? 2 : K <= 4 ? 4 : 8; }

// D == 0: 2-D data and [K][C][3][3] weights; D >= 1: 3-D data [N][D][H][W][C] and [K][C][3][3][3] weights
HeadArgs make(const void* h, int N, int D, int H, int W, int C, const float* pa, const float* pb, const float* w,
              int K) {
  HeadArgs A{};
  A.h = (const bf16r*)h;
  A.pa = pa;
  A.pb = pb;
  A.w = w;
  A.N = N; A.D = D > 0 ? D : 1; A.H = H; A.W = W; A.C = C; A.K = K; A.Kp = 8;
  A.T = D > 0 ? 27 : 9;
  A.tiles_x = W / HT;
  A.tiles_y = H / HT;
  A.ntiles = N * A.D * A.tiles_x * A.tiles_y;
  return A;
}

// 3-D: K <= 2 (the dgrad kernel keeps all 27 taps' weights of a 128-channel block in LDS)
bool shape_ok(int N, int D, int H, int W, int C, int K) {
  return N > 0 && D >= 0 && H % HT == 0 && W % HT == 0 && C % CK == 0 && K >= 1 && K <= (D > 0 ? 2 : 8) &&
         (long long)N * (D > 0 ? D : 1) * H * W * C < (1LL << 31);
}

constexpr int WG_WGRAD = 1024;  // head_wgrad workgroups (each loops over its share of tiles; 4 per CU at 256^2)
constexpr int RED_SPLIT = 32;   // first reduction stage: WG_WGRAD slots -> RED_SPLIT partial sums

// launch KERNEL<KT, KZ> for the runtime (K, D): KZ = 3 for 3-D (KT <= 2 there), 1 for 2-D
#define HEAD_LAUNCH(KERNEL, grid, A, st)                                                          \
  do {                                                                                            \
    if ((A).T == 27) {                                                                            \
      if (kt_of((A).K) == 1) hipLaunchKernelGGL((KERNEL<1, 3>), grid, dim3(NTH), 0, st, A);      \
      else hipLaunchKernelGGL((KERNEL<2, 3>), grid, dim3(NTH), 0, st, A);                         \
    } else {                                                                                      \
      switch (kt_of((A).K)) {                                                                     \
        case 1: hipLaunchKernelGGL((KERNEL<1, 1>), grid, dim3(NTH), 0, st, A); break;             \
        case 2: hipLaunchKernelGGL((KERNEL<2, 1>), grid, dim3(NTH), 0, st, A); break;             \
        case 4: hipLaunchKernelGGL((KERNEL<4, 1>), grid, dim3(NTH), 0, st, A); break;             \
        default: hipLaunchKernelGGL((KERNEL<8, 1>), grid, dim3(NTH), 0, st, A); break;            \
      }                                                                                           \
    }                                                                                             \
  } while (0)

}  // namespace

extern "C" {

int fmd_head_fwd(const void* h, int32_t N, int32_t D, int32_t H, int32_t W, int32_t C, const float* pro_a,
                 const float* pro_b, const float* w, const float* bias, int32_t K, float* out, fmd_stream_t s) {
  if (!shape_ok(N, D, H, W, C, K) || !pro_a || !pro_b) return -1;
  HeadArgs A = make(h, N, D, H, W, C, pro_a, pro_b, w, K);
  A.bias = bias;
  A.out = out;
  hipStream_t st = (hipStream_t)s;
  // chunk groups when the tiles alone leave most CUs idle (fewer than 128 tiles) and there are chunks to share
  const bool cg4 = A.ntiles < 128 && C >= 4 * CK;
#define FMD_HEAD_FWD(CGV)                                                                              \
  do {                                                                                                 \
    const dim3 g(A.ntiles), b(NTH * CGV);                                                              \
    if (A.T == 27) {                                                                                   \
      if (kt_of(K) == 1) hipLaunchKernelGGL((head_fwd<1, 3, CGV>), g, b, 0, st, A);                    \
      else hipLaunchKernelGGL((head_fwd<2, 3, CGV>), g, b, 0, st, A);                                  \
    } else {                                                                                           \
      switch (kt_of(K)) {                                                                              \
        case 1: hipLaunchKernelGGL((head_fwd<1, 1, CGV>), g, b, 0, st, A); break;                      \
        case 2: hipLaunchKernelGGL((head_fwd<2, 1, CGV>), g, b, 0, st, A); break;                      \
        case 4: hipLaunchKernelGGL((head_fwd<4, 1, CGV>), g, b, 0, st, A); break;                      \
        default: hipLaunchKernelGGL((head_fwd<8, 1, CGV>), g, b, 0, st, A); break;                     \
      }                                                                                                \
    }                                                                                                  \
  } while (0)
  if (cg4) FMD_HEAD_FWD(4);
  else FMD_HEAD_FWD(1);
#undef FMD_HEAD_FWD
  return (int)hipGetLastError();
}

int fmd_head_dgrad(const void* dpred, const float* w, int32_t K, const void* h, const float* pro_a, const float* pro_b,
                   int32_t N, int32_t D, int32_t H, int32_t W, int32_t C, void* dz, float* stats, fmd_stream_t s) {
  if (!shape_ok(N, D, H, W, C, K) || !pro_a || !pro_b || !stats) return -1;
  HeadArgs A = make(h, N, D, H, W, C, pro_a, pro_b, w, K);
  A.dpred = (const bf16r*)dpred;
  A.dz = (bf16r*)dz;
  A.stats = stats;
  hipStream_t st = (hipStream_t)s;
  HEAD_LAUNCH(head_dgrad, dim3(A.ntiles, (C + 127) / 128), A, st);
  return (int)hipGetLastError();
}

int64_t fmd_head_wgrad_workspace(int32_t N, int32_t D, int32_t H, int32_t W, int32_t C, int32_t K) {
  (void)N; (void)H; (void)W;
  const int kt = kt_of(K);
  return (int64_t)(WG_WGRAD + RED_SPLIT) * ((int64_t)kt * C * (D > 0 ? 27 : 9) + kt);
}

int fmd_head_wgrad(const void* dpred, int32_t K, const void* h, const float* pro_a, const float* pro_b, int32_t N,
                   int32_t D, int32_t H, int32_t W, int32_t C, float* dw, float* db, float* ws, fmd_stream_t s) {
  if (!shape_ok(N, D, H, W, C, K) || !pro_a || !pro_b || !ws || !dw) return -1;
  HeadArgs A = make(h, N, D, H, W, C, pro_a, pro_b, nullptr, K);
  A.dpred = (const bf16r*)dpred;
  A.ws = ws;
  const int nwg = A.ntiles < WG_WGRAD ? A.ntiles : WG_WGRAD;
  A.tiles_per_wg = (A.ntiles + nwg - 1) / nwg;
  const int kt = kt_of(K);
  hipStream_t st = (hipStream_t)s;
  HEAD_LAUNCH(head_wgrad, dim3(nwg), A, st);
  int rc = (int)hipGetLastError();
  if (rc) return rc;
  const int len = kt * C * A.T + kt;
  float* part = ws + (size_t)WG_WGRAD * len;
  const int per_split = (nwg + RED_SPLIT - 1) / RED_SPLIT;
  hipLaunchKernelGGL(slot_sum, dim3((len + 255) / 256, RED_SPLIT), dim3(256), 0, st, ws, nwg, (size_t)len, len,
                     per_split, part);
  rc = (int)hipGetLastError();
  if (rc) return rc;
  hipLaunchKernelGGL(head_wgrad_finish, dim3((len + 255) / 256), dim3(256), 0, st, part, RED_SPLIT, kt, K, C, A.T, dw,
                     db);
  return (int)hipGetLastError();
}

}  // extern "C"
