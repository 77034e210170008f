// Development probe: max |error| of three float NCO phasor forms against double sincospi, over a
// sweep of 32-bit phases P (phase = P / 2^32 cycles). Build:
//   hipcc -O3 --offload-arch=gfx950 tools/nco_accuracy.hip -o tools/nco_accuracy.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

__device__ float2 tab_poly(uint32_t P, const float2* tab) {
  const float2 h = tab[P >> 24];
  const float th = (float)(P & 0xFFFFFFu) * 0x1.921fb6p-30f;  // 2*pi / 2^32
  const float t2 = th * th;
  const float c = fmaf(t2, fmaf(t2, 1.0f / 24.0f, -0.5f), 1.0f);
  const float s = th * fmaf(t2, fmaf(t2, 1.0f / 120.0f, -1.0f / 6.0f), 1.0f);
  return make_float2(h.x * c - h.y * s, h.y * c + h.x * s);
}

__global__ void k_err(uint64_t count, uint32_t stride, unsigned long long* err_bits) {
  __shared__ float2 tab[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    float s, c;
    sincospif((float)(int8_t)i * 0x1p-7f, &s, &c);
    tab[i] = make_float2(c, s);
  }
  __syncthreads();
  double e0 = 0, e1 = 0, e2 = 0;
  for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < count; k += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t P = (uint32_t)(k * stride + (k >> 7));
    double sd, cd;
    sincospi((double)(int32_t)P * 0x1p-31, &sd, &cd);
    float s0, c0;
    sincospif((float)(int32_t)P * 0x1p-31f, &s0, &c0);
    const float x = (float)(int32_t)P * 0x1p-32f;
    const float s1 = __builtin_amdgcn_sinf(x), c1 = __builtin_amdgcn_cosf(x);
    const float2 t = tab_poly(P, tab);
    e0 = fmax(e0, fmax(fabs(s0 - sd), fabs(c0 - cd)));
    e1 = fmax(e1, fmax(fabs(s1 - sd), fabs(c1 - cd)));
    e2 = fmax(e2, fmax(fabs(t.y - sd), fabs(t.x - cd)));
  }
  atomicMax(&err_bits[0], (unsigned long long)__double_as_longlong(e0));
  atomicMax(&err_bits[1], (unsigned long long)__double_as_longlong(e1));
  atomicMax(&err_bits[2], (unsigned long long)__double_as_longlong(e2));
}

int main() {
  unsigned long long* d;
  (void)hipMalloc(&d, 3 * sizeof(unsigned long long));
  (void)hipMemset(d, 0, 3 * sizeof(unsigned long long));
  k_err<<<2048, 256>>>(1ull << 28, 16, d);
  unsigned long long h[3];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[3] = {"sincospif(float)", "v_sin/v_cos_f32", "table256+poly"};
  for (int i = 0; i < 3; ++i) {
    double e;
    memcpy(&e, &h[i], 8);
    printf("%-18s max abs err %.3e\n", names[i], e);
  }
  return 0;
}
