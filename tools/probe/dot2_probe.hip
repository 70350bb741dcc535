// Probe: v_dot2c_f32_bf16 (__builtin_amdgcn_fdot2_f32_bf16) vs the unpacked fp32 sum on random bf16 pairs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_;
__global__ void k(const unsigned* a, float* o) {
  const unsigned u = a[threadIdx.x];
  const bf16x2_ w = __builtin_bit_cast(bf16x2_, u);
  float s = 0.f, q = 0.f;
  for (int i = 0; i < 4; ++i) {
    s = __builtin_amdgcn_fdot2_f32_bf16(w, __builtin_bit_cast(bf16x2_, 0x3f803f80u), s, false);
    q = __builtin_amdgcn_fdot2_f32_bf16(w, w, q, false);
  }
  o[2 * threadIdx.x] = s;
  o[2 * threadIdx.x + 1] = q;
}
int main() {
  unsigned h[64];
  float r[128];
  srand(1);
  for (int i = 0; i < 64; ++i) h[i] = ((rand() & 0x7fff) + 0x3c00) | (((rand() & 0x7fff) + 0x3c00) << 16);
  unsigned* d; float* o;
  hipMalloc(&d, sizeof h); hipMalloc(&o, sizeof r);
  hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
  k<<<1, 64>>>(d, o);
  hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 64; ++i) {
    unsigned lo = h[i] << 16, hi = h[i] & 0xffff0000u;
    float a = *(float*)&lo, b = *(float*)&hi;
    float s = 4 * (a + b), q = 4 * (a * a + b * b);
    if (i < 4 || fabsf(r[2 * i] - s) > 1e-3f * fabsf(s) || fabsf(r[2 * i + 1] - q) > 1e-3f * fabsf(q)) {
      printf("%2d a=%g b=%g dot2 sum=%g (want %g) sq=%g (want %g)\n", i, a, b, r[2 * i], s, r[2 * i + 1], q);
      bad += i >= 4;
    }
  }
  printf("dot2 probe: %d mismatches\n", bad);
  return 0;
}
