// Probe: which (row, k-block) of A / (col, k-block) of B each lane's E8M0 scale
// of v_mfma_scale_f32_16x16x128_f8f6f4 applies to. All scales 127 (x1) except
// one lane's, set to 128 (x2); the change of C identifies the scaled sub-block.
// Prints, per lane, the matched (row|col, kblock) for A and for B, or "?".
// Build: hipcc --offload-arch=gfx950 -O2 -o mfma_scale_map mfma_scale_map.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

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
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, sa[l], 0, sb[l]);
  for (int i = 0; i < 4; ++i) C[(4 * (l >> 4) + i) * 16 + (l & 15)] = acc[i];
}

static float e4m3(unsigned char v) {
  const int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  float f = e == 0 ? std::ldexp((float)m / 8.f, -6) : std::ldexp(1.f + (float)m / 8.f, e - 7);
  return s ? -f : f;
}

int main() {
  unsigned char hA[16 * 128], hB[16 * 128];
  srand(11);
  for (int i = 0; i < 16 * 128; ++i) {
    unsigned char v;
    do { v = (unsigned char)(rand() & 0xff); } while (((v >> 3) & 15) > 9 || ((v >> 3) & 15) < 4);
    hA[i] = v;
    do { v = (unsigned char)(rand() & 0xff); } while (((v >> 3) & 15) > 9 || ((v >> 3) & 15) < 4);
    hB[i] = v;
  }
  // partial[r][c][kb] = sum over k in block kb of A[r][k] B[c][k]
  static double part[16][16][4];
  for (int r = 0; r < 16; ++r)
    for (int c = 0; c < 16; ++c)
      for (int kb = 0; kb < 4; ++kb) {
        double s = 0;
        for (int j = 0; j < 32; ++j) s += (double)e4m3(hA[r * 128 + 32 * kb + j]) * e4m3(hB[c * 128 + 32 * kb + j]);
        part[r][c][kb] = s;
      }
  unsigned char *dA, *dB;
  int *dsa, *dsb;
  float* dC;
  hipMalloc(&dA, sizeof hA);
  hipMalloc(&dB, sizeof hB);
  hipMalloc(&dsa, 256);
  hipMalloc(&dsb, 256);
  hipMalloc(&dC, 256 * 4);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  int ones[64];
  for (int l = 0; l < 64; ++l) ones[l] = 127;
  float base[256], pert[256];
  auto run = [&](const int* sa, const int* sb, float* out) {
    hipMemcpy(dsa, sa, 256, hipMemcpyHostToDevice);
    hipMemcpy(dsb, sb, 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC);
    hipMemcpy(out, dC, 1024, hipMemcpyDeviceToHost);
  };
  run(ones, ones, base);
  for (int which = 0; which < 2; ++which) {
    printf("%s scale: lane -> (%s, kblock)\n", which ? "B" : "A", which ? "col" : "row");
    for (int l = 0; l < 64; ++l) {
      int s[64];
      for (int i = 0; i < 64; ++i) s[i] = 127;
      s[l] = 128;
      run(which ? ones : s, which ? s : ones, pert);
      int found_x = -1, found_kb = -1, nz = 0;
      for (int i = 0; i < 256; ++i) nz += fabs(pert[i] - base[i]) > 1e-3;
      for (int x = 0; x < 16 && found_x < 0; ++x)
        for (int kb = 0; kb < 4; ++kb) {
          double err = 0;
          for (int r = 0; r < 16; ++r)
            for (int c = 0; c < 16; ++c) {
              const bool hit = which ? (c == x) : (r == x);
              const double want = hit ? part[r][c][kb] : 0.0;
              err = fmax(err, fabs((pert[r * 16 + c] - base[r * 16 + c]) - want));
            }
          if (err < 1e-2) {
            found_x = x;
            found_kb = kb;
            break;
          }
        }
      if (found_x >= 0) printf(" %d:(%d,%d)", l, found_x, found_kb);
      else printf(" %d:?(nz=%d)", l, nz);
    }
    printf("\n");
  }
  return 0;
}
