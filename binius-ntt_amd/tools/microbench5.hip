// Dev microbenchmark (not part of the library): VALU issue rate per instruction form -- VGPR source
// banks (bank = index mod 4), SGPR/inline-constant operands, DPP, v_bfe/v_perm/v_cndmask -- at 1-4
// waves per SIMD. Build: hipcc -O3 --offload-arch=gfx950 microbench5.hip -o /tmp/mb5
#include <hip/hip_runtime.h>
#include <stdio.h>
#define R4(a,b,c,d) a "\n" b "\n" c "\n" d "\n"
#define REP8(x) x x x x x x x x
#define CLOB "v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v16","v20","v24","v28","v32","v36"
#define KERNEL(name, body) \
__global__ __launch_bounds__(256) void name(unsigned* out, int iters) { \
  for (int i = 0; i < iters; i++) { asm volatile(REP8(body) ::: CLOB); } \
  if (threadIdx.x == 1000) out[0] = 1; }
// 4 instructions per body, dests v8..v11 (banks 0..3)
KERNEL(k_xor_diff, R4("v_xor_b32 v8, v1, v2","v_xor_b32 v9, v1, v2","v_xor_b32 v10, v1, v2","v_xor_b32 v11, v1, v2"))
KERNEL(k_xor_same, R4("v_xor_b32 v8, v4, v12","v_xor_b32 v9, v4, v12","v_xor_b32 v10, v4, v12","v_xor_b32 v11, v4, v12"))
KERNEL(k_b3_diff, R4("v_bitop3_b32 v8, v1, v2, v3 bitop3:0x96","v_bitop3_b32 v9, v1, v2, v3 bitop3:0x96","v_bitop3_b32 v10, v1, v2, v3 bitop3:0x96","v_bitop3_b32 v11, v1, v2, v3 bitop3:0x96"))
KERNEL(k_b3_two, R4("v_bitop3_b32 v8, v4, v12, v1 bitop3:0x96","v_bitop3_b32 v9, v4, v12, v1 bitop3:0x96","v_bitop3_b32 v10, v4, v12, v1 bitop3:0x96","v_bitop3_b32 v11, v4, v12, v1 bitop3:0x96"))
KERNEL(k_b3_two_b, R4("v_bitop3_b32 v8, v1, v4, v12 bitop3:0x96","v_bitop3_b32 v9, v1, v4, v12 bitop3:0x96","v_bitop3_b32 v10, v1, v4, v12 bitop3:0x96","v_bitop3_b32 v11, v1, v4, v12 bitop3:0x96"))
KERNEL(k_b3_same, R4("v_bitop3_b32 v8, v4, v12, v16 bitop3:0x96","v_bitop3_b32 v9, v4, v12, v16 bitop3:0x96","v_bitop3_b32 v10, v4, v12, v16 bitop3:0x96","v_bitop3_b32 v11, v4, v12, v16 bitop3:0x96"))
KERNEL(k_b3_dup, R4("v_bitop3_b32 v8, v1, v1, v2 bitop3:0x6a","v_bitop3_b32 v9, v1, v1, v2 bitop3:0x6a","v_bitop3_b32 v10, v1, v1, v2 bitop3:0x6a","v_bitop3_b32 v11, v1, v1, v2 bitop3:0x6a"))
KERNEL(k_b3_sgpr, R4("v_bitop3_b32 v8, s4, v1, v2 bitop3:0x6a","v_bitop3_b32 v9, s4, v1, v2 bitop3:0x6a","v_bitop3_b32 v10, s4, v1, v2 bitop3:0x6a","v_bitop3_b32 v11, s4, v1, v2 bitop3:0x6a"))
// dest always bank 0 with sources in banks 1,2,3
KERNEL(k_b3_dst0, R4("v_bitop3_b32 v8, v1, v2, v3 bitop3:0x96","v_bitop3_b32 v12, v1, v2, v3 bitop3:0x96","v_bitop3_b32 v16, v1, v2, v3 bitop3:0x96","v_bitop3_b32 v20, v1, v2, v3 bitop3:0x96"))
// mixed: 2 xor + 2 bitop3, conflict free
KERNEL(k_mix, R4("v_xor_b32 v8, v1, v2","v_bitop3_b32 v9, v1, v2, v3 bitop3:0x96","v_xor_b32 v10, v5, v6","v_bitop3_b32 v11, v5, v6, v7 bitop3:0x96"))
// dependent chains with fresh results as sources (typical circuit): chain over v8..v11
KERNEL(k_b3_dep_diff, R4("v_bitop3_b32 v9, v8, v2, v3 bitop3:0x96","v_bitop3_b32 v10, v9, v3, v1 bitop3:0x96","v_bitop3_b32 v11, v10, v1, v2 bitop3:0x96","v_bitop3_b32 v8, v11, v5, v6 bitop3:0x96"))
KERNEL(k_bfe, R4("v_bfe_i32 v8, v1, 3, 1","v_bfe_i32 v9, v1, 4, 1","v_bfe_i32 v10, v1, 5, 1","v_bfe_i32 v11, v1, 6, 1"))
KERNEL(k_bfe_v, R4("v_bfe_i32 v8, v1, v2, v3","v_bfe_i32 v9, v1, v2, v3","v_bfe_i32 v10, v1, v2, v3","v_bfe_i32 v11, v1, v2, v3"))
KERNEL(k_xor_s, R4("v_xor_b32 v8, s4, v1","v_xor_b32 v9, s4, v1","v_xor_b32 v10, s4, v1","v_xor_b32 v11, s4, v1"))
KERNEL(k_b3_k, R4("v_bitop3_b32 v8, v1, v2, 1 bitop3:0x6a","v_bitop3_b32 v9, v1, v2, 1 bitop3:0x6a","v_bitop3_b32 v10, v1, v2, 1 bitop3:0x6a","v_bitop3_b32 v11, v1, v2, 1 bitop3:0x6a"))

KERNEL(k_xor_e64, R4("v_xor_b32_e64 v8, v1, v2","v_xor_b32_e64 v9, v1, v2","v_xor_b32_e64 v10, v1, v2","v_xor_b32_e64 v11, v1, v2"))
KERNEL(k_lsh, R4("v_lshrrev_b32 v8, 3, v1","v_lshrrev_b32 v9, 3, v1","v_lshrrev_b32 v10, 3, v1","v_lshrrev_b32 v11, 3, v1"))
KERNEL(k_perm, R4("v_perm_b32 v8, v1, v2, v3","v_perm_b32 v9, v1, v2, v3","v_perm_b32 v10, v1, v2, v3","v_perm_b32 v11, v1, v2, v3"))
KERNEL(k_cnd, R4("v_cndmask_b32_e64 v8, 0, v1, s[4:5]","v_cndmask_b32_e64 v9, 0, v1, s[4:5]","v_cndmask_b32_e64 v10, 0, v1, s[4:5]","v_cndmask_b32_e64 v11, 0, v1, s[4:5]"))
KERNEL(k_and_dpp, R4("v_and_b32_dpp v8, v1, v2 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf","v_and_b32_dpp v9, v1, v2 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf","v_and_b32_dpp v10, v1, v2 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf","v_and_b32_dpp v11, v1, v2 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf"))
int main() {
  unsigned* out; hipMalloc(&out, 64);
  int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int iters = 40000; const double ipi = 8 * 4;
  struct K { const char* n; void (*f)(unsigned*, int); } ks[] = {
    {"xor 2 banks", k_xor_diff}, {"xor same bank", k_xor_same}, {"b3 3 banks", k_b3_diff},
    {"b3 src0,1 same bank", k_b3_two}, {"b3 src1,2 same bank", k_b3_two_b}, {"b3 all same bank", k_b3_same},
    {"b3 dup reg", k_b3_dup}, {"b3 sgpr+2 banks", k_b3_sgpr}, {"b3 dst bank0", k_b3_dst0}, {"mix xor/b3", k_mix},
    {"b3 dep chain diff", k_b3_dep_diff}, {"bfe", k_bfe}, {"bfe vgpr", k_bfe_v}, {"xor sgpr", k_xor_s}, {"b3 inline const", k_b3_k}, {"xor e64", k_xor_e64}, {"lshr", k_lsh}, {"perm", k_perm}, {"cndmask sgpr", k_cnd}, {"and dpp", k_and_dpp}};
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int w = 0; w < 3; w++) hipLaunchKernelGGL(k_b3_diff, dim3(cus*2), dim3(256), 0, 0, out, iters);
  hipDeviceSynchronize();
  for (auto& k : ks) {
    printf("%-22s", k.n);
    for (int wps = 1; wps <= 4; wps++) {
      const int grid = cus * wps;
      hipLaunchKernelGGL(k.f, dim3(grid), dim3(256), 0, 0, out, iters);
      hipEventRecord(a);
      hipLaunchKernelGGL(k.f, dim3(grid), dim3(256), 0, 0, out, iters);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms = 0; hipEventElapsedTime(&ms, a, b);
      const double inst = (double)grid * 4 * iters * ipi;
      printf("  %.3f", inst / (ms * 1e-3) / (cus * 4.0) / 2.4e9);
    }
    printf("   (wave-instr per SIMD-cycle @2.4GHz, 1..4 waves/SIMD)\n");
  }
  return 0;
}
