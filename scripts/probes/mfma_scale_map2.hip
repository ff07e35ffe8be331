// Probe 2 for v_mfma_scale_f32_16x16x128_f8f6f4 scale semantics with
// structured data: A = 1 on k-block q only (q = 0..3, 32 K each), B = 1.
// For each lane l with its scale set to x2 (others x1), print which C elements
// change (as the row or column index they share) and, per q, whether the
// change appears - i.e. which (row|col, k-block) each lane's scale covers.
#include <hip/hip_runtime.h>

#include <cstdio>

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

int main() {
  const unsigned char ONE = 0x38;  // e4m3 1.0
  unsigned char hA[16 * 128], hB[16 * 128];
  unsigned char *dA, *dB;
  int *dsa, *dsb;
  float* dC;
  (void)hipMalloc(&dA, sizeof hA);
  (void)hipMalloc(&dB, sizeof hB);
  (void)hipMalloc(&dsa, 256);
  (void)hipMalloc(&dsb, 256);
  (void)hipMalloc(&dC, 1024);
  for (int i = 0; i < 16 * 128; ++i) hB[i] = ONE;
  (void)hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  for (int which = 0; which < 2; ++which) {
    printf("%s scale:\n", which ? "B" : "A");
    for (int l = 0; l < 64; ++l) {
      printf(" lane %2d:", l);
      for (int q = 0; q < 4; ++q) {
        for (int r = 0; r < 16; ++r)
          for (int kk = 0; kk < 128; ++kk) hA[r * 128 + kk] = (kk / 32 == q) ? ONE : 0;
        if (which) {  // probe B: put the structure on B instead
          for (int i = 0; i < 16 * 128; ++i) { unsigned char t = hA[i]; hA[i] = ONE; hB[i] = t; }
        }
        (void)hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
        (void)hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
        int s1[64], s2[64];
        for (int i = 0; i < 64; ++i) s1[i] = s2[i] = 127;
        (which ? s2 : s1)[l] = 128;
        (void)hipMemcpy(dsa, s1, 256, hipMemcpyHostToDevice);
        (void)hipMemcpy(dsb, s2, 256, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC);
        float C[256];
        (void)hipMemcpy(C, dC, 1024, hipMemcpyDeviceToHost);
        // changed elements: value != 32
        int rows = 0, cols = 0, n = 0;
        for (int r = 0; r < 16; ++r)
          for (int c = 0; c < 16; ++c)
            if (C[r * 16 + c] != 32.f) { rows |= 1 << r; cols |= 1 << c; ++n; }
        if (n) printf(" q%d:n%d r%04x c%04x v%.0f", q, n, rows, cols, C[__builtin_ctz(rows) * 16 + __builtin_ctz(cols)]);
        if (which) for (int i = 0; i < 16 * 128; ++i) hB[i] = ONE;
      }
      printf("\n");
    }
  }
  return 0;
}
