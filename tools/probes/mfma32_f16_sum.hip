// Probe: v_mfma_f32_32x32x16_f16 (gfx950) -- operand / result lane maps and
// how it sums K, for the x3 density's 32x32 layout (abc_mvn_x3.hip):
//   1. layout: random small-integer A, B, C (every product and sum exact)
//      against D[i][j] = C[i][j] + sum_k A[i][k] B[k][j] with
//      A[row l&31][k 8(l>>5)+e], B[k 8(l>>5)+e][col l&31],
//      D: col l&31, row (r&3) + 8(r>>2) + 4(l>>5);
//   2. exact block: 12 products that are multiples of a grid g with every
//      partial sum below 2^24 g, plus C (a multiple of g) -- must be exact;
//   3. grouping: big terms in K 0..7 and tiny ones in K 8..15 with C
//      cancelling the big ones (two sequential 8-groups keep the tiny sum),
//      and the reverse order;
//   4. lo block: after an exact first MFMA leaves |acc| ~ 1, a second MFMA
//      of class-1/class-2-sized products; error vs exact relative to 2^-24.
//   hipcc -O2 --offload-arch=gfx950 mfma32_f16_sum.hip -o mfma32_f16_sum
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// A [32][16] row-major, B [16][32] row-major, C/D [32][32] row-major; two
// chained MFMAs when A2/B2 are given (D = A2 B2 + (A B + C))
__global__ void probe(const float* A, const float* B, const float* A2, const float* B2,
                      const float* C, float* D) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  half8 a, b, a2, b2;
  for (int e = 0; e < 8; ++e) {
    a[e] = (_Float16)A[r * 16 + 8 * h + e];
    b[e] = (_Float16)B[(8 * h + e) * 32 + r];
    a2[e] = A2 ? (_Float16)A2[r * 16 + 8 * h + e] : (_Float16)0.f;
    b2[e] = B2 ? (_Float16)B2[(8 * h + e) * 32 + r] : (_Float16)0.f;
  }
  f32x16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = C[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r];
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
  if (A2) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a2, b2, acc, 0, 0, 0);
  for (int i = 0; i < 16; ++i) D[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = acc[i];
}

static float *dA, *dB, *dA2, *dB2, *dC, *dD;

static void run(const float* A, const float* B, const float* A2, const float* B2,
                const float* C, float* D) {
  hipMemcpy(dA, A, 32 * 16 * 4, hipMemcpyHostToDevice);
  hipMemcpy(dB, B, 16 * 32 * 4, hipMemcpyHostToDevice);
  if (A2) {
    hipMemcpy(dA2, A2, 32 * 16 * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB2, B2, 16 * 32 * 4, hipMemcpyHostToDevice);
  }
  hipMemcpy(dC, C, 32 * 32 * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, A2 ? dA2 : nullptr,
                     A2 ? dB2 : nullptr, dC, dD);
  hipMemcpy(D, dD, 32 * 32 * 4, hipMemcpyDeviceToHost);
}

static double exact(const float* A, const float* B, const float* A2, const float* B2,
                    const float* C, int i, int j) {
  double s = C[i * 32 + j];
  for (int k = 0; k < 16; ++k) s += (double)A[i * 16 + k] * (double)B[k * 32 + j];
  if (A2)
    for (int k = 0; k < 16; ++k) s += (double)A2[i * 16 + k] * (double)B2[k * 32 + j];
  return s;
}

static double urand() { return rand() / (RAND_MAX + 1.0); }

int main() {
  hipMalloc(&dA, 4096); hipMalloc(&dB, 4096); hipMalloc(&dA2, 4096); hipMalloc(&dB2, 4096);
  hipMalloc(&dC, 4096); hipMalloc(&dD, 4096);
  float A[512], B[512], A2[512], B2[512], C[1024], D[1024];
  srand(7);
  // 1. layout
  {
    for (int q = 0; q < 512; ++q) { A[q] = (float)(rand() % 17 - 8); B[q] = (float)(rand() % 17 - 8); }
    for (int q = 0; q < 1024; ++q) C[q] = (float)(rand() % 2001 - 1000);
    run(A, B, nullptr, nullptr, C, D);
    int bad = 0;
    for (int i = 0; i < 32; ++i)
      for (int j = 0; j < 32; ++j) bad += (double)D[i * 32 + j] != exact(A, B, nullptr, nullptr, C, i, j);
    printf("layout: %d of 1024 entries differ from C + A B\n", bad);
  }
  // 2. exact block: grid g = 2^-10; coordinate limbs |a|, |b| <= 647 (sum of
  //    the 10 products <= 2^22 g, as |z||y| <= 2^2E in x3), 10 coordinate products + 2 scalar limbs, C =
  //    an integer multiple of g, 2000 trials over the 1024 entries
  {
    long bad = 0, tot = 0;
    double maxrel = 0;
    for (int trial = 0; trial < 200; ++trial) {
      for (int i = 0; i < 32; ++i)
        for (int k = 0; k < 16; ++k) {
          const int v = k < 10 ? (rand() % 1295) - 647 : (k < 12 ? (rand() % 4097) - 2048 : 0);
          A[i * 16 + k] = ldexpf((float)v, k < 10 ? 0 : 1);
        }
      for (int k = 0; k < 16; ++k)
        for (int j = 0; j < 32; ++j) {
          const int v = (rand() % 1295) - 647;
          B[k * 32 + j] = k < 10 ? ldexpf((float)v, -10) : (k < 12 ? ldexpf(1.f, k == 10 ? 0 : -11) : 0.f);
        }
      for (int q = 0; q < 1024; ++q) C[q] = ldexpf((float)((rand() % 8388607) - 4194303), -10);
      run(A, B, nullptr, nullptr, C, D);
      for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
          const double ex = exact(A, B, nullptr, nullptr, C, i, j);
          ++tot;
          if ((double)D[i * 32 + j] != ex) {
            ++bad;
            const double rel = fabs(D[i * 32 + j] - ex) / fmax(fabs(ex), 1e-30);
            if (rel > maxrel) maxrel = rel;
          }
        }
    }
    printf("exact block: %ld of %ld entries not exact (max rel %.3e)\n", bad, tot, maxrel);
  }
  // 3. grouping
  {
    const float tiny = ldexpf(1.f, -10);
    for (int order = 0; order < 2; ++order) {
      for (int q = 0; q < 512; ++q) { A[q] = 0.f; B[q] = 0.f; }
      for (int q = 0; q < 1024; ++q) C[q] = 0.f;
      for (int k = 0; k < 16; ++k) {
        const bool big = order == 0 ? k < 8 : k >= 8;
        A[k] = big ? 2048.f : tiny;
        B[k * 32] = big ? 1024.f : tiny * 3;
      }
      C[0] = -ldexpf(1.f, 24);   // -(8 * 2^21)
      run(A, B, nullptr, nullptr, C, D);
      printf("grouping (%s): got % .9e exact % .9e\n",
             order == 0 ? "big K0-7, tiny K8-15" : "tiny K0-7, big K8-15", D[0],
             exact(A, B, nullptr, nullptr, C, 0, 0));
    }
  }
  // 4. lo block after an exact block
  {
    double maxerr = 0, maxacc = 0;
    for (int trial = 0; trial < 100; ++trial) {
      for (int i = 0; i < 32; ++i)
        for (int k = 0; k < 16; ++k) {
          A[i * 16 + k] = k < 2 ? (float)((rand() % 4097) - 2048) : 0.f;
          A2[i * 16 + k] = ldexpf((float)((rand() % 2049) - 1024), -5);
        }
      for (int k = 0; k < 16; ++k)
        for (int j = 0; j < 32; ++j) {
          B[k * 32 + j] = k < 2 ? (float)((rand() % 4097) - 2048) : 0.f;
          B2[k * 32 + j] = ldexpf((float)((rand() % 2049) - 1024), -(int)(10 + 11 * urand()));
        }
      for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
          double s = 0;
          for (int k = 0; k < 2; ++k) s += (double)A[i * 16 + k] * (double)B[k * 32 + j];
          C[i * 32 + j] = (float)(-s + (rand() % 5) - 2);   // exact block leaves -2..2
        }
      run(A, B, A2, B2, C, D);
      for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
          const double ex = exact(A, B, A2, B2, C, i, j);
          maxerr = fmax(maxerr, fabs(D[i * 32 + j] - ex));
          maxacc = fmax(maxacc, fabs(ex));
        }
    }
    printf("lo block after exact block: max |err| %.3e (2^%.1f), max |acc| %.3e\n", maxerr,
           log2(maxerr > 0 ? maxerr : 1e-300), maxacc);
  }
  return 0;
}
