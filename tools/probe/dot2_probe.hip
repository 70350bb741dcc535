// probe: semantics of v_dot2c_f32_bf16 on gfx950 (a.lo*b.lo + a.hi*b.hi + c)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
__global__ void k(const unsigned* a, const unsigned* b, const float* c, float* o) {
  int i = threadIdx.x;
  o[i] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, a[i]), __builtin_bit_cast(bf16x2, b[i]), c[i], false);
}
static unsigned bf(float f) { unsigned u; memcpy(&u, &f, 4); return u >> 16; }
int main() {
  const int n = 4;
  float av[n][2] = {{1, 2}, {3, -1}, {0.5f, 4}, {2, 0}}, bv[n][2] = {{1, 1}, {2, 5}, {2, 0.25f}, {0, 7}}, cv[n] = {0, 1, 10, -3};
  unsigned ha[n], hb[n];
  for (int i = 0; i < n; ++i) { ha[i] = bf(av[i][0]) | bf(av[i][1]) << 16; hb[i] = bf(bv[i][0]) | bf(bv[i][1]) << 16; }
  unsigned *da, *db; float *dc, *dout;
  hipMalloc(&da, 16); hipMalloc(&db, 16); hipMalloc(&dc, 16); hipMalloc(&dout, 16);
  hipMemcpy(da, ha, 16, hipMemcpyHostToDevice); hipMemcpy(db, hb, 16, hipMemcpyHostToDevice);
  hipMemcpy(dc, cv, 16, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(n), 0, 0, da, db, dc, dout);
  float out[n];
  hipMemcpy(out, dout, 16, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; ++i)
    printf("got %g want %g\n", out[i], av[i][0] * bv[i][0] + av[i][1] * bv[i][1] + cv[i]);
  return 0;
}
