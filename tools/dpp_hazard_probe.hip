// Probe: does a DPP read of a VGPR need more than the generic 2 wait states when the VGPR was
// written by a packed-fp32 VALU op (v_pk_add/mul/fma_f32) on gfx950?  And does a packed-fp32 read
// of a DPP result need any?  (Round-3 evidence: the fused norm3 of xattn_block_kernel<320,40>,
// built with SLP vectorisation, fed v_mov_b32_dpp from v_pk_add_f32 results at exactly 2 wait
// states and corrupted one 16-lane pass in ~1e-7 of those DPP reads; profiles/r3_xattn_determinism.txt.)
//
// Each variant runs one fixed instruction sequence in inline asm (so the spacing is exactly what the
// string says) and checks every lane's result bitwise against the same value moved by ds_bpermute.
// Build: hipcc --offload-arch=gfx950 -O3 tools/dpp_hazard_probe.hip -o tools/build/dpp_hazard_probe
// Run:   tools/build/dpp_hazard_probe [iters] [reps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

#define DPP_SWAP " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"

// pattern A: VALU write of v41 -> <spacing> -> v_mov_b32_dpp reading v41 (lane ^ 1)
#define PAT_A(WRITE, SPACING)                                                                        \
  asm volatile(WRITE SPACING "v_mov_b32_dpp %0, v41" DPP_SWAP "s_nop 1\n"                           \
               : "=v"(r) : "v"(x), "v"(y) : "v40", "v41")
// pattern A on the low half (v40)
#define PAT_A_LO(WRITE, SPACING)                                                                     \
  asm volatile(WRITE SPACING "v_mov_b32_dpp %0, v40" DPP_SWAP "s_nop 1\n"                           \
               : "=v"(r) : "v"(x), "v"(y) : "v40", "v41")
// pattern B: v_mov_b32_dpp writes v40 / v41 -> <spacing> -> VALU read of v[40:41]
#define PAT_B(READ, SPACING)                                                                         \
  asm volatile("s_nop 4\n"                                                                           \
               "v_mov_b32_dpp v41, %1" DPP_SWAP "v_mov_b32_dpp v40, %2" DPP_SWAP SPACING READ "s_nop 1\n" \
               : "=v"(r2) : "v"(x[1]), "v"(x[0]), "v"(y) : "v40", "v41")

#define W_ADD "v_add_f32 v41, %1, %2\n"          // scalar: v41 = x.lo + y.lo (operands printed as pairs: use halves below)
#define W_PK_ADD "v_pk_add_f32 v[40:41], %1, %2\n"
#define W_PK_MUL "v_pk_mul_f32 v[40:41], %1, %2\n"
#define W_PK_FMA "v_pk_fma_f32 v[40:41], %1, %2, %1\n"
#define R_PK_ADD "v_pk_add_f32 %0, v[40:41], %3\n"
#define R_ADD "v_add_f32 %0, v41, %3\n"

#define S1 "s_nop 0\n"
#define S2 "s_nop 1\n"
#define S3 "s_nop 2\n"
#define S4 "s_nop 3\n"
#define S5 "s_nop 4\n"

constexpr int NV = 18;
static const char* kNames[NV] = {
    "A  v_add_f32      -> dpp  1 ws (below spec: control)",
    "A  v_add_f32      -> dpp  2 ws",
    "A  v_pk_add_f32   -> dpp  1 ws (below spec)",
    "A  v_pk_add_f32   -> dpp  2 ws (the SLP norm3 sequence)",
    "A  v_pk_add_f32   -> dpp  3 ws",
    "A  v_pk_add_f32   -> dpp  4 ws",
    "A  v_pk_add_f32   -> dpp  5 ws",
    "A  v_pk_mul_f32   -> dpp  2 ws",
    "A  v_pk_fma_f32   -> dpp  2 ws",
    "A  v_pk_add_f32 lo-> dpp  2 ws",
    "B  dpp -> v_pk_add_f32 0 ws",
    "B  dpp -> v_pk_add_f32 1 ws",
    "B  dpp -> v_pk_add_f32 2 ws",
    "B  dpp -> v_add_f32    0 ws",
    "A  v_pk_add_f32   -> dpp  2 ws, v_mov between (compiled form)",
    "A  v_add_f32      -> dpp  3 ws",
    "C  SLP quad reduction (v_pk_add_f32 <-> v_mov_b32_dpp pairs)",
    "D  op_sel:[0,1] op_sel_hi:[1,0] v_pk_add_f32 (semantics check, no DPP)",
};

__device__ float* g_dbg = nullptr;   // one wave's lanes: x, y, result, expected (dump mode)

template <int V>
__device__ __forceinline__ bool run_one(f2 x, f2 y) {
  const int lane = threadIdx.x & 63;
  (void)lane;
  if constexpr (V == 16) {
    // the quad reduction of ln_quad_stats as the SLP build emitted it (round-3 xattn.hip ISA, norm3 epilogue):
    // a pair (lo, hi) summed over the 4 lanes of a quad with two v_mov_b32_dpp per step into a register pair,
    // the 'old' operand copied from a zero register that the second step then overwrites
    f2 r2;
    asm volatile(
        "v_mov_b32 v44, 0\n"
        "v_mov_b32 v43, v44\n"
        "v_pk_add_f32 v[40:41], %1, %2\n"
        "v_mov_b32 v42, v44\n"
        "s_nop 0\n"
        "v_mov_b32_dpp v43, v41" DPP_SWAP
        "v_mov_b32_dpp v42, v40" DPP_SWAP
        "v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n"
        "v_mov_b32 v43, v44\n"
        "v_mov_b32 v45, v44\n"
        "v_mov_b32_dpp v44, v40 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
        "v_mov_b32_dpp v43, v41 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
        "v_mov_b32 v42, v44\n"
        "v_pk_add_f32 %0, v[40:41], v[42:43]\n"
        "s_nop 1\n"
        : "=v"(r2) : "v"(x), "v"(y) : "v40", "v41", "v42", "v43", "v44", "v45");
    const float a = x[0] + y[0], b = x[1] + y[1];
    const float a1 = a + __shfl_xor(a, 1, 64), b1 = b + __shfl_xor(b, 1, 64);
    const float a2 = a1 + __shfl_xor(a1, 2, 64), b2 = b1 + __shfl_xor(b1, 2, 64);
    if (g_dbg) {
      float* d = g_dbg + 8 * lane;
      d[0] = x[0]; d[1] = x[1]; d[2] = y[0]; d[3] = y[1]; d[4] = r2[0]; d[5] = r2[1]; d[6] = a2; d[7] = b2;
    }
    return (__builtin_bit_cast(unsigned, r2[0]) != __builtin_bit_cast(unsigned, a2)) |
           (__builtin_bit_cast(unsigned, r2[1]) != __builtin_bit_cast(unsigned, b2));
  } else if constexpr (V == 17) {
    f2 r2;
    asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0]\n" "s_nop 1\n" : "=v"(r2) : "v"(x), "v"(y));
    if (g_dbg) {
      float* d = g_dbg + 8 * lane;
      d[0] = x[0]; d[1] = x[1]; d[2] = y[0]; d[3] = y[1]; d[4] = r2[0]; d[5] = r2[1]; d[6] = x[0] + y[1]; d[7] = x[1] + y[0];
    }
    return (__builtin_bit_cast(unsigned, r2[0]) != __builtin_bit_cast(unsigned, x[0] + y[1])) |
           (__builtin_bit_cast(unsigned, r2[1]) != __builtin_bit_cast(unsigned, x[1] + y[0]));
  } else if constexpr (V <= 9 || V == 14 || V == 15) {
    float r;
    float e;
    if constexpr (V == 0 || V == 1 || V == 15) {
      // scalar writer: v41 = x.y + y.y
      const float xa = x[1], ya = y[1];
      if constexpr (V == 0)
        asm volatile("v_add_f32 v41, %1, %2\n" S1 "v_mov_b32_dpp %0, v41" DPP_SWAP "s_nop 1\n" : "=v"(r) : "v"(xa), "v"(ya) : "v41");
      else if constexpr (V == 1)
        asm volatile("v_add_f32 v41, %1, %2\n" S2 "v_mov_b32_dpp %0, v41" DPP_SWAP "s_nop 1\n" : "=v"(r) : "v"(xa), "v"(ya) : "v41");
      else
        asm volatile("v_add_f32 v41, %1, %2\n" S3 "v_mov_b32_dpp %0, v41" DPP_SWAP "s_nop 1\n" : "=v"(r) : "v"(xa), "v"(ya) : "v41");
      e = __shfl_xor(x[1] + y[1], 1, 64);
    } else if constexpr (V == 2) { PAT_A(W_PK_ADD, S1); e = __shfl_xor(x[1] + y[1], 1, 64);
    } else if constexpr (V == 3) { PAT_A(W_PK_ADD, S2); e = __shfl_xor(x[1] + y[1], 1, 64);
    } else if constexpr (V == 4) { PAT_A(W_PK_ADD, S3); e = __shfl_xor(x[1] + y[1], 1, 64);
    } else if constexpr (V == 5) { PAT_A(W_PK_ADD, S4); e = __shfl_xor(x[1] + y[1], 1, 64);
    } else if constexpr (V == 6) { PAT_A(W_PK_ADD, S5); e = __shfl_xor(x[1] + y[1], 1, 64);
    } else if constexpr (V == 7) { PAT_A(W_PK_MUL, S2); e = __shfl_xor(x[1] * y[1], 1, 64);
    } else if constexpr (V == 8) { PAT_A(W_PK_FMA, S2); e = __shfl_xor(__builtin_fmaf(x[1], y[1], x[1]), 1, 64);
    } else if constexpr (V == 9) { PAT_A_LO(W_PK_ADD, S2); e = __shfl_xor(x[0] + y[0], 1, 64);
    } else {  // V == 14: v_mov of an unrelated register between the write and the read, as the compiler emitted it
      asm volatile("v_pk_add_f32 v[40:41], %1, %2\n" "v_mov_b32 v42, v40\n" "s_nop 0\n"
                   "v_mov_b32_dpp %0, v41" DPP_SWAP "s_nop 1\n" : "=v"(r) : "v"(x), "v"(y) : "v40", "v41", "v42");
      e = __shfl_xor(x[1] + y[1], 1, 64);
    }
    return __builtin_bit_cast(unsigned, r) != __builtin_bit_cast(unsigned, e);
  } else {
    f2 r2;
    f2 e2;
    if constexpr (V == 10) { PAT_B(R_PK_ADD, "");
    } else if constexpr (V == 11) { PAT_B(R_PK_ADD, S1);
    } else if constexpr (V == 12) { PAT_B(R_PK_ADD, S2);
    } else {
      float r1;
      const float yb = y[1];
      asm volatile("s_nop 4\n" "v_mov_b32_dpp v41, %1" DPP_SWAP R_ADD "s_nop 1\n" : "=v"(r1) : "v"(x[1]), "v"(0.f), "v"(yb) : "v41");
      r2 = f2{0.f, r1};
    }
    if constexpr (V == 13) {
      e2 = f2{0.f, __shfl_xor(x[1], 1, 64) + y[1]};
    } else {
      e2 = f2{__shfl_xor(x[0], 1, 64) + y[0], __shfl_xor(x[1], 1, 64) + y[1]};
    }
    return (__builtin_bit_cast(unsigned, r2[0]) != __builtin_bit_cast(unsigned, e2[0])) |
           (__builtin_bit_cast(unsigned, r2[1]) != __builtin_bit_cast(unsigned, e2[1]));
  }
}

// Waves [0, load_waves) of each workgroup run a dependent MFMA chain (the UNet's kernels keep the
// matrix pipe busy while other waves issue VALU); the rest run the probe.
template <int V>
__global__ void __launch_bounds__(256) probe_kernel(unsigned long long* errs, int iters, int load_waves, float* sink) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __shared__ __attribute__((aligned(16))) h8 lds[4][64 * 8];
  if (wave < -load_waves) {
    // LDS + global-store load (the fused block's epilogue: ds_read / ds_write of row chunks, 16-B stores)
    h8 v = {};
    for (int i = 0; i < iters / 8; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) lds[wave][j * 64 + lane] = v;
      __builtin_amdgcn_s_waitcnt(0xc07f);
#pragma unroll
      for (int j = 0; j < 8; ++j) v += lds[wave][((j + 1) & 7) * 64 + lane];
      reinterpret_cast<h8*>(sink + 256)[((blockIdx.x * 4 + wave) * 64 + lane) & 0xFFFF] = v;
    }
    if ((float)v[0] == 12345.f) sink[threadIdx.x] = (float)v[1];
    return;
  }
  if (wave < load_waves) {
    h8 a, b;
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] = (_Float16)(0.001f * (lane + j)); b[j] = (_Float16)(0.002f * (j - lane)); }
    f16v acc = {};
    for (int i = 0; i < iters / 4; ++i) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, acc, 0, 0, 0);
    }
    if (acc[0] == 12345.f) sink[threadIdx.x] = acc[1];
    return;
  }
  f2 x = {lane * 0.37f + blockIdx.x * 0.001f, lane * 1.13f - wave * 0.5f};
  f2 y = {0.25f * wave + 1.0f, 3.0f + 0.01f * lane};
  unsigned bad = 0;
  for (int i = 0; i < iters; ++i) {
    bad += run_one<V>(x, y) ? 1u : 0u;
    x[0] += 1.0f;
    x[1] += 0.5f;
    y[1] -= 0.25f;
  }
  if (bad) atomicAdd(errs + V, (unsigned long long)bad);
}

template <int V>
void launch(unsigned long long* errs, int iters, int load_waves, float* sink, int blocks) {
  hipLaunchKernelGGL(probe_kernel<V>, dim3(blocks), dim3(256), 0, 0, errs, iters, load_waves, sink);
}

template <int... Vs>
void launch_all(int v, unsigned long long* errs, int iters, int lw, float* sink, int blocks, std::integer_sequence<int, Vs...>) {
  ((v == Vs ? launch<Vs>(errs, iters, lw, sink, blocks) : void()), ...);
}

template <int V>
__global__ void dump_kernel(float* out) {
  g_dbg = out;
  const int lane = threadIdx.x & 63;
  f2 x = {lane * 0.37f, lane * 1.13f};
  f2 y = {1.0f, 3.0f + 0.01f * lane};
  run_one<V>(x, y);
}

int main(int argc, char** argv) {
  if (argc > 1 && argv[1][0] == 'd') {   // dump mode: variants 16 / 17, one wave, lanes 0-7
    float* d;
    hipMalloc(&d, 64 * 8 * sizeof(float));
    float h[64 * 8];
    hipLaunchKernelGGL(dump_kernel<16>, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("variant 16: lane x.lo x.hi y.lo y.hi | asm lo hi | expected lo hi\n");
    for (int l = 0; l < 8; ++l) printf("  %2d %9.4f %9.4f %9.4f %9.4f | %10.4f %10.4f | %10.4f %10.4f\n", l, h[8*l], h[8*l+1], h[8*l+2], h[8*l+3], h[8*l+4], h[8*l+5], h[8*l+6], h[8*l+7]);
    hipLaunchKernelGGL(dump_kernel<17>, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("variant 17:\n");
    for (int l = 0; l < 8; ++l) printf("  %2d %9.4f %9.4f %9.4f %9.4f | %10.4f %10.4f | %10.4f %10.4f\n", l, h[8*l], h[8*l+1], h[8*l+2], h[8*l+3], h[8*l+4], h[8*l+5], h[8*l+6], h[8*l+7]);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
  }
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  const int reps = argc > 2 ? atoi(argv[2]) : 4;
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int blocks = prop.multiProcessorCount * 8;
  unsigned long long* errs;
  float* sink;
  hipMalloc(&errs, NV * sizeof(unsigned long long));
  hipMalloc(&sink, 256 * sizeof(float) + 65536 * 16);
  printf("%s, %d CUs, %d workgroups x 4 waves, %d iterations per wave, %d reps per load mode\n", prop.gcnArchName,
         prop.multiProcessorCount, blocks, iters, reps);
  for (int lw : {0, 2, -2}) {   // -2: two LDS / store load waves per workgroup
    hipMemset(errs, 0, NV * sizeof(unsigned long long));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float ms_total = 0.f;
    for (int rep = 0; rep < reps; ++rep)
      for (int v = 0; v < NV; ++v) {
        hipEventRecord(e0);
        launch_all(v, errs, iters, lw, sink, blocks, std::make_integer_sequence<int, NV>{});
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms_total += ms;
      }
    unsigned long long h[NV];
    hipMemcpy(h, errs, sizeof(h), hipMemcpyDeviceToHost);
    const double checks = (double)reps * blocks * (4 - (lw < 0 ? -lw : lw)) * 64 * iters;
    printf("\n-- %d %s load waves per workgroup (%.0f ms); lane-checks per variant %.3e\n", lw < 0 ? -lw : lw,
           lw < 0 ? "LDS/store" : "MFMA", ms_total, checks);
    for (int v = 0; v < NV; ++v) printf("  %-62s mismatching lanes %llu (%.2e)\n", kNames[v], h[v], h[v] / checks);
  }
  hipError_t st = hipDeviceSynchronize();
  printf("\nstatus %s\n", hipGetErrorString(st));
  return st == hipSuccess ? 0 : 1;
}
