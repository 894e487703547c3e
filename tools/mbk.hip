// Main-loop variants on one workgroup, to separate MFMA, load and loop costs (GPU box).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mbk.hip -o build/mbk
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e = (x);                                                                    \
    if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); }        \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma4(f32x4 a, f32x4 b, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
  return acc;
}
__device__ __forceinline__ f32x4 ld(__amdgpu_buffer_rsrc_t r, int off) {
  u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return f32x4{__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
}

// MODE 0: MFMA only; 1: loads only (summed); 2: loads + MFMA ring 4; 3: ring 8;
// 4: loads only, blocked layout (each load = one contiguous 1 KB block); 5: MODE 1 twice over the same data
template <int MODE>
__global__ __launch_bounds__(256) void k(const float* A, const float* B, float* out, int K) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = lane & 15, rl = 4 * (lane >> 4);
  __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, 0x7fff0000, 0x00020000);
  __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, 0, 0x7fff0000, 0x00020000);
  int oa = (row * K + rl) * 4, ob = ((wave * 16 + row) * K + rl) * 4;
  const int nch = K / 16;
  f32x4 acc0 = {0, 0, 0, 0}, acc1 = acc0;
  if (MODE == 0) {
    f32x4 a = {A[lane], 1.f, 2.f, 3.f}, b = {B[lane], 1.f, 1.f, 1.f};
    for (int c = 0; c < nch; c += 2) {
      acc0 = mfma4(a, b, acc0);
      acc1 = mfma4(b, a, acc1);
    }
  } else if (MODE == 4) {
    // blocked: A block (chunk c) at c*1KB, B block for wave w at (w*nch + c)*1KB
    int pa = lane * 16, pb = (wave * nch) * 1024 + lane * 16;
    f32x4 a0 = ld(ra, pa), b0 = ld(rb, pb), a1 = ld(ra, pa + 1024), b1 = ld(rb, pb + 1024);
    f32x4 a2 = ld(ra, pa + 2048), b2 = ld(rb, pb + 2048), a3 = ld(ra, pa + 3072), b3 = ld(rb, pb + 3072);
    pa += 4096; pb += 4096;
#pragma unroll 1
    for (int c = 0; c < nch; c += 4) {
      acc0 += a0 * b0; a0 = ld(ra, pa); b0 = ld(rb, pb);
      acc1 += a1 * b1; a1 = ld(ra, pa + 1024); b1 = ld(rb, pb + 1024);
      acc0 += a2 * b2; a2 = ld(ra, pa + 2048); b2 = ld(rb, pb + 2048);
      acc1 += a3 * b3; a3 = ld(ra, pa + 3072); b3 = ld(rb, pb + 3072);
      pa += 4096; pb += 4096;
    }
  } else if (MODE == 6 || MODE == 7) {
    // A lane-linear blocks; B "strided use" of a blocked tensor: lane (col c = l&15, g = l>>4)
    // reads rows 4g..4g+3 of column c -> 4 dwords at ((c>>2)*64 + (4g+j)*4 + (c&3))*4 bytes
    const int c = lane & 15, g = lane >> 4;
    int pa = lane * 16, pb = (wave * nch) * 1024 + (((c >> 2) * 64 + 16 * g + (c & 3)) * 4);
    for (int pass = 0; pass < (MODE == 7 ? 2 : 1); ++pass) {
      int qa = pa, qb = pb;
#pragma unroll 1
      for (int ch = 0; ch < nch; ch += 2) {
        f32x4 a0 = ld(ra, qa), a1 = ld(ra, qa + 1024);
        f32x4 b0, b1;
        b0.x = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, qb, 0, 0));
        b0.y = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, qb + 16, 0, 0));
        b0.z = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, qb + 32, 0, 0));
        b0.w = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, qb + 48, 0, 0));
        b1.x = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, qb + 1024, 0, 0));
        b1.y = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, qb + 1040, 0, 0));
        b1.z = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, qb + 1056, 0, 0));
        b1.w = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, qb + 1072, 0, 0));
        acc0 = mfma4(a0, b0, acc0);
        acc1 = mfma4(a1, b1, acc1);
        qa += 2048; qb += 2048;
      }
    }
  } else if (MODE == 8 || MODE == 9) {
    // ring-4 pipelined: MODE 8 = A lane-linear + B strided-use; MODE 9 = both strided-use
    const int c = lane & 15, g = lane >> 4;
    const int so = ((c >> 2) * 64 + 16 * g + (c & 3)) * 4;
    int pa = (MODE == 9 ? so : lane * 16), pb = (wave * nch) * 1024 + so;
    auto LA = [&](int off) {
      if (MODE == 8) return ld(ra, off);
      f32x4 v;
      v.x = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ra, off, 0, 0));
      v.y = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ra, off + 16, 0, 0));
      v.z = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ra, off + 32, 0, 0));
      v.w = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ra, off + 48, 0, 0));
      return v;
    };
    auto LB = [&](int off) {
      f32x4 v;
      v.x = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, off, 0, 0));
      v.y = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, off + 16, 0, 0));
      v.z = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, off + 32, 0, 0));
      v.w = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, off + 48, 0, 0));
      return v;
    };
    f32x4 a0 = LA(pa), b0 = LB(pb), a1 = LA(pa + 1024), b1 = LB(pb + 1024);
    f32x4 a2 = LA(pa + 2048), b2 = LB(pb + 2048), a3 = LA(pa + 3072), b3 = LB(pb + 3072);
    pa += 4096; pb += 4096;
#pragma unroll 1
    for (int ch = 0; ch < nch; ch += 4) {
      acc0 = mfma4(a0, b0, acc0); a0 = LA(pa); b0 = LB(pb);
      acc1 = mfma4(a1, b1, acc1); a1 = LA(pa + 1024); b1 = LB(pb + 1024);
      acc0 = mfma4(a2, b2, acc0); a2 = LA(pa + 2048); b2 = LB(pb + 2048);
      acc1 = mfma4(a3, b3, acc1); a3 = LA(pa + 3072); b3 = LB(pb + 3072);
      pa += 4096; pb += 4096;
    }
  } else if (MODE == 10) {
    // blocked lane-linear both, ring 4, with MFMA
    int pa = lane * 16, pb = (wave * nch) * 1024 + lane * 16;
    f32x4 a0 = ld(ra, pa), b0 = ld(rb, pb), a1 = ld(ra, pa + 1024), b1 = ld(rb, pb + 1024);
    f32x4 a2 = ld(ra, pa + 2048), b2 = ld(rb, pb + 2048), a3 = ld(ra, pa + 3072), b3 = ld(rb, pb + 3072);
    pa += 4096; pb += 4096;
#pragma unroll 1
    for (int ch = 0; ch < nch; ch += 4) {
      acc0 = mfma4(a0, b0, acc0); a0 = ld(ra, pa); b0 = ld(rb, pb);
      acc1 = mfma4(a1, b1, acc1); a1 = ld(ra, pa + 1024); b1 = ld(rb, pb + 1024);
      acc0 = mfma4(a2, b2, acc0); a2 = ld(ra, pa + 2048); b2 = ld(rb, pb + 2048);
      acc1 = mfma4(a3, b3, acc1); a3 = ld(ra, pa + 3072); b3 = ld(rb, pb + 3072);
      pa += 4096; pb += 4096;
    }
  } else if (MODE == 5) {
    for (int pass = 0; pass < 2; ++pass) {
      int qa = oa, qb = ob;
      f32x4 a0 = ld(ra, qa), b0 = ld(rb, qb), a1 = ld(ra, qa + 64), b1 = ld(rb, qb + 64);
      qa += 128; qb += 128;
#pragma unroll 1
      for (int c = 0; c < nch; c += 2) {
        acc0 += a0 * b0; a0 = ld(ra, qa); b0 = ld(rb, qb);
        acc1 += a1 * b1; a1 = ld(ra, qa + 64); b1 = ld(rb, qb + 64);
        qa += 128; qb += 128;
      }
    }
  } else if (MODE == 1 || MODE == 2) {
    f32x4 a0 = ld(ra, oa), b0 = ld(rb, ob), a1 = ld(ra, oa + 64), b1 = ld(rb, ob + 64);
    f32x4 a2 = ld(ra, oa + 128), b2 = ld(rb, ob + 128), a3 = ld(ra, oa + 192), b3 = ld(rb, ob + 192);
    oa += 256; ob += 256;
#pragma unroll 1
    for (int c = 0; c < nch; c += 4) {
      if (MODE == 1) acc0 += a0 * b0; else acc0 = mfma4(a0, b0, acc0);
      a0 = ld(ra, oa); b0 = ld(rb, ob);
      if (MODE == 1) acc1 += a1 * b1; else acc1 = mfma4(a1, b1, acc1);
      a1 = ld(ra, oa + 64); b1 = ld(rb, ob + 64);
      if (MODE == 1) acc0 += a2 * b2; else acc0 = mfma4(a2, b2, acc0);
      a2 = ld(ra, oa + 128); b2 = ld(rb, ob + 128);
      if (MODE == 1) acc1 += a3 * b3; else acc1 = mfma4(a3, b3, acc1);
      a3 = ld(ra, oa + 192); b3 = ld(rb, ob + 192);
      oa += 256; ob += 256;
    }
  } else {
    f32x4 a[8], b[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) { a[q] = ld(ra, oa + 64 * q); b[q] = ld(rb, ob + 64 * q); }
    oa += 512; ob += 512;
#pragma unroll 1
    for (int c = 0; c < nch; c += 8) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (q & 1) acc1 = mfma4(a[q], b[q], acc1); else acc0 = mfma4(a[q], b[q], acc0);
        a[q] = ld(ra, oa + 64 * q); b[q] = ld(rb, ob + 64 * q);
      }
      oa += 512; ob += 512;
    }
  }
  f32x4 r = acc0 + acc1;
  out[threadIdx.x] = r.x + r.y + r.z + r.w;
}

template <int MODE>
static double timeit(const float* A, const float* B, float* o, int K, int nwg, hipStream_t st) {
  const int reps = 100;
  hipGraph_t g;
  hipGraphExec_t x;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k<MODE>, dim3(nwg), dim3(256), 0, st, A, B, o, K);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(x, st));
  CK(hipStreamSynchronize(st));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, st));
  CK(hipGraphLaunch(x, st));
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGraphExecDestroy(x));
  CK(hipGraphDestroy(g));
  return ms * 1000.0 / reps;
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  float *A, *B, *o;
  CK(hipMalloc(&A, 64 << 20));
  CK(hipMalloc(&B, 64 << 20));
  CK(hipMalloc(&o, 1 << 20));
  CK(hipMemset(A, 0, 64 << 20));
  CK(hipMemset(B, 0, 64 << 20));
  const char* names[] = {"mfma only", "loads only (r4)", "loads+mfma r4", "loads+mfma r8", "blocked loads", "2 passes"};
  for (int K : {64, 256, 1024, 4096}) {
    printf("K=%5d:", K);
    printf("  %s %7.2f", names[0], timeit<0>(A, B, o, K, 1, st));
    printf("  %s %7.2f", names[1], timeit<1>(A, B, o, K, 1, st));
    printf("  %s %7.2f", names[2], timeit<2>(A, B, o, K, 1, st));
    printf("  %s %7.2f", names[3], timeit<3>(A, B, o, K, 1, st));
    printf("  %s %7.2f", names[4], timeit<4>(A, B, o, K, 1, st));
    printf("  %s %7.2f", names[5], timeit<5>(A, B, o, K, 1, st));
    printf("  strided-use %7.2f  x2 %7.2f us\n", timeit<6>(A, B, o, K, 1, st), timeit<7>(A, B, o, K, 1, st));
    printf("         ring4+mfma: lin/lin %7.2f  lin/strided %7.2f  strided/strided %7.2f us\n",
           timeit<10>(A, B, o, K, 1, st), timeit<8>(A, B, o, K, 1, st), timeit<9>(A, B, o, K, 1, st));
  }
  for (int K : {256, 1024}) {
    for (int nwg : {8, 64, 256, 1024}) {
      printf("K=%5d nwg=%4d: loads(r4) %7.2f  blocked %7.2f us\n", K, nwg, timeit<1>(A, B, o, K, nwg, st),
             timeit<4>(A, B, o, K, nwg, st));
    }
  }
  return 0;
}
