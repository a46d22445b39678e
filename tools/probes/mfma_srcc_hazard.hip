// Dependent-MFMA and MFMA->VALU timing on gfx950, VGPR-form accumulators
// (build with -mllvm -amdgpu-mfma-vgpr-form, as abc_mvn_x3.hip is):
//  * chain  : producer MFMA (16x16x32 f16 or 16x16x16 f16) -> G wait states
//             -> consumer MFMA taking the producer's result as SrcC;
//  * valu   : producer MFMA -> G wait states -> v_add reading its result.
// G = -1 leaves the schedule to the compiler (no asm); otherwise an
// `asm volatile` of s_nops totalling G wait states is tied to the result
// ("+v"), so nothing else sits between.  Small integer operands: every
// result is exact; the reference sums the separate products on the VALU.
// Prints the number of wrong lanes per case.  tools/probes only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int G, typename T>
__device__ __forceinline__ void gap2(f32x4& r, T& x) {
  if constexpr (G == 0) asm volatile("" : "+v"(r), "+v"(x));
  if constexpr (G == 1) asm volatile("s_nop 0" : "+v"(r), "+v"(x));
  if constexpr (G == 2) asm volatile("s_nop 1" : "+v"(r), "+v"(x));
  if constexpr (G == 3) asm volatile("s_nop 2" : "+v"(r), "+v"(x));
  if constexpr (G == 4) asm volatile("s_nop 3" : "+v"(r), "+v"(x));
  if constexpr (G == 6) asm volatile("s_nop 5" : "+v"(r), "+v"(x));
  if constexpr (G == 8) asm volatile("s_nop 7" : "+v"(r), "+v"(x));
  if constexpr (G == 10) asm volatile("s_nop 7\n\ts_nop 1" : "+v"(r), "+v"(x));
  if constexpr (G == 12) asm volatile("s_nop 7\n\ts_nop 3" : "+v"(r), "+v"(x));
  if constexpr (G == 16) asm volatile("s_nop 7\n\ts_nop 7" : "+v"(r), "+v"(x));
  if constexpr (G == 20) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+v"(r), "+v"(x));
  if constexpr (G == 24) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(r), "+v"(x));
}

template <int G>
__device__ __forceinline__ void gap(f32x4& r) {
  if constexpr (G == 0) asm volatile("" : "+v"(r));
  if constexpr (G == 1) asm volatile("s_nop 0" : "+v"(r));
  if constexpr (G == 2) asm volatile("s_nop 1" : "+v"(r));
  if constexpr (G == 3) asm volatile("s_nop 2" : "+v"(r));
  if constexpr (G == 4) asm volatile("s_nop 3" : "+v"(r));
  if constexpr (G == 6) asm volatile("s_nop 5" : "+v"(r));
  if constexpr (G == 8) asm volatile("s_nop 7" : "+v"(r));
  if constexpr (G == 10) asm volatile("s_nop 7\n\ts_nop 1" : "+v"(r));
  if constexpr (G == 12) asm volatile("s_nop 7\n\ts_nop 3" : "+v"(r));
  if constexpr (G == 16) asm volatile("s_nop 7\n\ts_nop 7" : "+v"(r));
  if constexpr (G == 20) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+v"(r));
  if constexpr (G == 24) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(r));
}

template <int S>
__device__ __forceinline__ f32x4 mm(half8 a, half8 b, half4 a4, half4 b4, f32x4 c) {
  if constexpr (S == 32) return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c, 0, 0, 0);
}

// MODE 0: chain P -> G -> Q (SrcC); MODE 1: P -> G -> v_add;
// MODE 2: P -> G -> independent Q (own accumulator from 0), both read
template <int MODE, int P, int Q, int G>
__global__ void probe(const half8* A, const half8* B, const half4* A4, const half4* B4,
                      float* out) {
  const int lane = threadIdx.x;
  half8 a = A[lane], b = B[lane], a2 = A[64 + lane], b2 = B[64 + lane];
  half4 a4 = A4[lane], b4 = B4[lane], a42 = A4[64 + lane], b42 = B4[64 + lane];
  // every operand in registers (loads waited for) before the producer issues
  asm volatile("" : "+v"(a), "+v"(b), "+v"(a2), "+v"(b2), "+v"(a4), "+v"(b4), "+v"(a42),
               "+v"(b42));
  half8 ra = a, rb = b, ra2 = a2, rb2 = b2;
  half4 ra4 = a4, rb4 = b4, ra42 = a42, rb42 = b42;
  asm volatile("" : "+v"(ra), "+v"(rb), "+v"(ra2), "+v"(rb2), "+v"(ra4), "+v"(rb4),
               "+v"(ra42), "+v"(rb42));   // the reference's copies (no CSE)
  f32x4 r = mm<P>(a, b, a4, b4, f32x4{0.f, 0.f, 0.f, 0.f});
  if constexpr (MODE == 2) {
    if constexpr (Q == 32) gap2<G>(r, a2); else gap2<G>(r, a42);
    f32x4 r2 = mm<Q>(a2, b2, a42, b42, f32x4{0.f, 0.f, 0.f, 0.f});
    r += r2;
  } else {
    gap<G>(r);
  }
  if (MODE == 0) r = mm<Q>(a2, b2, a42, b42, r);
  f32x4 v;
  for (int i = 0; i < 4; ++i) v[i] = r[i] + 1.0f;
  for (int i = 0; i < 4; ++i) out[lane * 4 + i] = v[i];
  // reference: separate products, summed on the VALU after a full drain
  f32x4 p = mm<P>(ra, rb, ra4, rb4, f32x4{0.f, 0.f, 0.f, 0.f});
  f32x4 q = MODE != 1 ? mm<Q>(ra2, rb2, ra42, rb42, f32x4{0.f, 0.f, 0.f, 0.f})
                      : f32x4{0.f, 0.f, 0.f, 0.f};
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(p), "+v"(q));
  for (int i = 0; i < 4; ++i) out[256 + lane * 4 + i] = (p[i] + q[i]) + 1.0f;
}

template <int MODE, int P, int Q, int G>
void run(half8* A, half8* B, half4* A4, half4* B4, float* d_out) {
  hipLaunchKernelGGL((probe<MODE, P, Q, G>), dim3(1), dim3(64), 0, 0, A, B, A4, B4, d_out);
  std::vector<float> h(512);
  (void)hipMemcpy(h.data(), d_out, 512 * sizeof(float), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 256; ++i) bad += h[i] != h[256 + i];
  if (MODE == 0)
    printf("chain x%d -> x%d  gap %3d: %3d / 256 wrong\n", P, Q, G, bad);
  else if (MODE == 2)
    printf("indep x%d -> x%d  gap %3d: %3d / 256 wrong\n", P, Q, G, bad);
  else
    printf("valu  x%d -> add  gap %3d: %3d / 256 wrong\n", P, G, bad);
}

template <int MODE, int P, int Q>
void sweep(half8* A, half8* B, half4* A4, half4* B4, float* o) {
  run<MODE, P, Q, -1>(A, B, A4, B4, o); run<MODE, P, Q, 0>(A, B, A4, B4, o);
  run<MODE, P, Q, 1>(A, B, A4, B4, o);  run<MODE, P, Q, 2>(A, B, A4, B4, o);
  run<MODE, P, Q, 3>(A, B, A4, B4, o);  run<MODE, P, Q, 4>(A, B, A4, B4, o);
  run<MODE, P, Q, 6>(A, B, A4, B4, o);  run<MODE, P, Q, 8>(A, B, A4, B4, o);
  run<MODE, P, Q, 10>(A, B, A4, B4, o); run<MODE, P, Q, 12>(A, B, A4, B4, o);
  run<MODE, P, Q, 16>(A, B, A4, B4, o); run<MODE, P, Q, 20>(A, B, A4, B4, o);
  run<MODE, P, Q, 24>(A, B, A4, B4, o);
}

int main() {
  std::vector<_Float16> a(128 * 8), b(128 * 8), a4(128 * 4), b4(128 * 4);
  for (int i = 0; i < 128 * 8; ++i) { a[i] = (_Float16)(i % 7 - 3); b[i] = (_Float16)(i % 5 - 2); }
  for (int i = 0; i < 128 * 4; ++i) { a4[i] = (_Float16)(i % 3 + 1); b4[i] = (_Float16)(i % 11 - 5); }
  half8 *A, *B;
  half4 *A4, *B4;
  float* out;
  (void)hipMalloc(&A, 128 * 16); (void)hipMalloc(&B, 128 * 16);
  (void)hipMalloc(&A4, 128 * 8); (void)hipMalloc(&B4, 128 * 8);
  (void)hipMalloc(&out, 512 * 4);
  (void)hipMemcpy(A, a.data(), 128 * 16, hipMemcpyHostToDevice);
  (void)hipMemcpy(B, b.data(), 128 * 16, hipMemcpyHostToDevice);
  (void)hipMemcpy(A4, a4.data(), 128 * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(B4, b4.data(), 128 * 8, hipMemcpyHostToDevice);
  sweep<0, 32, 32>(A, B, A4, B4, out);
  sweep<0, 32, 16>(A, B, A4, B4, out);
  sweep<0, 16, 32>(A, B, A4, B4, out);
  sweep<0, 16, 16>(A, B, A4, B4, out);
  sweep<2, 32, 16>(A, B, A4, B4, out);
  sweep<2, 16, 32>(A, B, A4, B4, out);
  sweep<1, 32, 0>(A, B, A4, B4, out);
  sweep<1, 16, 0>(A, B, A4, B4, out);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
