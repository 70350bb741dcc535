// Launch arguments of the halo-tiled 3x3 stride-1 convolution kernels (csrc/conv_halo.hip, csrc/conv_halo9.hip).
#pragma once
#include "common.h"
#include "../../include/fmdiff.h"

struct HArgs {
  fmd_conv_desc d;
  int C, C23;
  int tiles_x, tiles_y, ntc;
  int nchunk1, nchunk2;   // main / 1x1-segment chunks
  int splits, cps;        // split-K over main chunks: split y owns chunks [y*cps, min(nchunk1, (y+1)*cps));
                          // the 1x1 segment belongs to the last split; fp32 partials go to d.ws
  int nsteps_slots;       // taps over the whole reduction (9 per 3x3 chunk + 1 per 1x1 chunk)
  const bf16r* wt;        // pre-tiled main weights [ntc][nchunk1][9][KC][BCO][8]
  const bf16r* wt2;       // pre-tiled 1x1 weights  [ntc][nchunk2][KC][BCO][8]
  int depth, ncb, dsrc;   // 3-D (depth > 0): images are the N*depth output slices; main chunk = (depth tap
                          // kz, 32-channel block cb) = kz*ncb + cb, reading logical input slice z + kz - 1
                          // (zeros outside; stored slice >> 1 under nearest-x2, dsrc = stored depth);
                          // per-sample tables (GN affine, bias_nc, ep_a/b) are indexed by slice / depth
  unsigned long long* tbuf;    // per-wave phase timestamps (compiled in only with -DFMD_HALO_TIME)
  int fold_E0, fold_E1;        // d.fold_st0: statistics slab rows per image of src0 / src1
  double fold_inv;             // 1 / (channels per group x pixels per image)
  int dbg;                     // debug ablations (fmd_debug_halo_flags; compiled in only with -DFMD_HALO_DBG):
                               // 1 no halo loads, 2 no transform, 4 no epilogue, 8 no weight DMA in the loop,
                               // 16 no SiLU' in the epilogue, 32 no statistics, 64 no side-tile loads
};

// v9 kernel (csrc/conv_halo9.hip): launches the problem A describes if it qualifies; returns 1 (not applicable),
// 0 (launched) or a hipError_t.  pro: 0 raw input, 1 GroupNorm affine, 2 affine + SiLU.
int halo9_launch(const HArgs& A, int pro, fmd_stream_t stream);
