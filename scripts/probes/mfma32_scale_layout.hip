// Probe: v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3) operand/result layout and
// per-row scales. Hypothesis: lane l holds A[row l&31][k = 32*(l>>5) + j] and
// B[k = 32*(l>>5) + j][col l&31], j = 0..31; C/D as 32x32x16 bf16:
// col = l&31, row = (reg&3) + 8*(reg>>2) + 4*(l>>5). Row scale: every lane
// with l&31 == r carries row r's E8M0 scale (scale_a), column scale likewise.
// Prints the max abs error vs a host reference with per-row / per-col scales.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

__global__ void k(const unsigned char* A, const unsigned char* B, const int* sr, const int* sc, float* C) {
  const int l = threadIdx.x;
  v8i a, b;
  unsigned char* pa = reinterpret_cast<unsigned char*>(&a);
  unsigned char* pb = reinterpret_cast<unsigned char*>(&b);
  for (int j = 0; j < 32; ++j) {
    const int kk = 32 * (l >> 5) + j;
    pa[j] = A[(l & 31) * 64 + kk];
    pb[j] = B[(l & 31) * 64 + kk];
  }
  f16v acc = {};
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, 0, 0, 0, sr[l & 31], 0, sc[l & 31]);
  for (int r = 0; r < 16; ++r) C[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = acc[r];
}

static float e4m3(unsigned char v) {
  const int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  float f = e == 0 ? std::ldexp((float)m / 8.f, -6) : std::ldexp(1.f + (float)m / 8.f, e - 7);
  return s ? -f : f;
}

int main() {
  unsigned char hA[32 * 64], hB[32 * 64];
  int hr[32], hc[32];
  srand(3);
  for (int i = 0; i < 32 * 64; ++i) {
    unsigned char v;
    do { v = (unsigned char)(rand() & 0xff); } while (((v >> 3) & 15) > 9 || ((v >> 3) & 15) < 4);
    hA[i] = v;
    do { v = (unsigned char)(rand() & 0xff); } while (((v >> 3) & 15) > 9 || ((v >> 3) & 15) < 4);
    hB[i] = v;
  }
  for (int i = 0; i < 32; ++i) {
    hr[i] = 124 + rand() % 7;
    hc[i] = 124 + rand() % 7;
  }
  unsigned char *dA, *dB;
  int *dr, *dc;
  float* dC;
  (void)hipMalloc(&dA, sizeof hA);
  (void)hipMalloc(&dB, sizeof hB);
  (void)hipMalloc(&dr, sizeof hr);
  (void)hipMalloc(&dc, sizeof hc);
  (void)hipMalloc(&dC, 1024 * 4);
  (void)hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  (void)hipMemcpy(dr, hr, sizeof hr, hipMemcpyHostToDevice);
  (void)hipMemcpy(dc, hc, sizeof hc, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dr, dc, dC);
  float hC[1024];
  (void)hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
  double err = 0, mx = 0;
  for (int r = 0; r < 32; ++r)
    for (int c = 0; c < 32; ++c) {
      double s = 0;
      for (int kk = 0; kk < 64; ++kk) s += (double)e4m3(hA[r * 64 + kk]) * e4m3(hB[c * 64 + kk]);
      s *= std::ldexp(1.0, hr[r] - 127) * std::ldexp(1.0, hc[c] - 127);
      err = fmax(err, fabs(s - hC[r * 32 + c]));
      mx = fmax(mx, fabs(s));
    }
  printf("32x32x64 scaled fp8: max|C| %.3f max err %.3e (%s)\n", mx, err, err < 1e-3 * mx ? "layout OK" : "MISMATCH");
  return 0;
}
