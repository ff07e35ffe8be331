// Probe: semantics of the E8M0 scale operands of
// v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3). Hypothesis H1: lane l's
// scale_a applies to A[row l&15][k-block l>>4] (32 K each), lane l's scale_b to
// B[k-block l>>4][col l&15]; opsel selects the byte of the 32-bit scale VGPR.
// H2 (alternative): lanes 0-15 hold one scale per row for all 128 K.
// Prints the max relative error of the MFMA result against both hypotheses
// for opsel 0 and for opsel 1 (scale moved to byte 1).
// Build: hipcc --offload-arch=gfx950 -O2 -o mfma_scale_semantics mfma_scale_semantics.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int OPSEL>
__global__ void k(const unsigned char* A, const unsigned char* B, const int* sa, const int* sb, float* C) {
  const int l = threadIdx.x;
  v8i a, b;
  unsigned char* pa = reinterpret_cast<unsigned char*>(&a);
  unsigned char* pb = reinterpret_cast<unsigned char*>(&b);
  for (int j = 0; j < 32; ++j) {
    const int kk = 32 * (l >> 4) + j;
    pa[j] = A[(l & 15) * 128 + kk];
    pb[j] = B[(l & 15) * 128 + kk];
  }
  f4 acc = {0, 0, 0, 0};
  const int xa = sa[l] << (8 * OPSEL), xb = sb[l] << (8 * OPSEL);
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, OPSEL, xa, OPSEL, xb);
  for (int i = 0; i < 4; ++i) C[(4 * (l >> 4) + i) * 16 + (l & 15)] = acc[i];
}

static float e4m3(unsigned char v) {
  const int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  float f = e == 0 ? std::ldexp((float)m / 8.f, -6) : std::ldexp(1.f + (float)m / 8.f, e - 7);
  return s ? -f : f;
}

int main() {
  unsigned char hA[16 * 128], hB[16 * 128];
  int hsa[64], hsb[64];
  srand(7);
  for (int i = 0; i < 16 * 128; ++i) {
    unsigned char v;
    do { v = (unsigned char)(rand() & 0xff); } while (((v >> 3) & 15) > 9 || ((v >> 3) & 15) < 4);
    hA[i] = v;
    do { v = (unsigned char)(rand() & 0xff); } while (((v >> 3) & 15) > 9 || ((v >> 3) & 15) < 4);
    hB[i] = v;
  }
  for (int l = 0; l < 64; ++l) {
    hsa[l] = 124 + rand() % 7;
    hsb[l] = 124 + rand() % 7;
  }
  unsigned char *dA, *dB;
  int *dsa, *dsb;
  float* dC;
  hipMalloc(&dA, sizeof hA);
  hipMalloc(&dB, sizeof hB);
  hipMalloc(&dsa, sizeof hsa);
  hipMalloc(&dsb, sizeof hsb);
  hipMalloc(&dC, 256 * 4);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipMemcpy(dsa, hsa, sizeof hsa, hipMemcpyHostToDevice);
  hipMemcpy(dsb, hsb, sizeof hsb, hipMemcpyHostToDevice);
  for (int opsel = 0; opsel < 2; ++opsel) {
    if (opsel == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC);
    else hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC);
    float hC[256];
    hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
    double e1 = 0, e2 = 0, mx = 0;
    for (int r = 0; r < 16; ++r)
      for (int c = 0; c < 16; ++c) {
        double h1 = 0, h2 = 0;
        for (int kk = 0; kk < 128; ++kk) {
          const int kb = kk / 32;
          const double p = (double)e4m3(hA[r * 128 + kk]) * e4m3(hB[c * 128 + kk]);
          h1 += p * std::ldexp(1.0, hsa[kb * 16 + r] - 127) * std::ldexp(1.0, hsb[kb * 16 + c] - 127);
          h2 += p * std::ldexp(1.0, hsa[r] - 127) * std::ldexp(1.0, hsb[c] - 127);
        }
        const double g = hC[r * 16 + c];
        e1 = fmax(e1, fabs(g - h1));
        e2 = fmax(e2, fabs(g - h2));
        mx = fmax(mx, fabs(h1));
      }
    printf("opsel %d: max|C| %.3f  err H1 (lane=row|kblock<<4) %.3e  err H2 (lanes 0-15 per row) %.3e\n", opsel, mx,
           e1, e2);
  }
  return 0;
}
