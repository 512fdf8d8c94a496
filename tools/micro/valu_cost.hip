// valu_cost.hip -- issue cost (cycles per wave-instruction) of the VALU instructions of the dense
// draw on gfx950: one wave per SIMD, 8 independent chains of one instruction, unrolled; prints
// cycles per instruction from s_memtime. Build: hipcc --offload-arch=gfx950 -O3 -o valu_cost valu_cost.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(X) X X X X X X X X
#define BODY(INS)                                                                                         \
    asm volatile(REP8(INS " v[0:1], v[2:3], v[4:5]\n\t" INS " v[6:7], v[8:9], v[10:11]\n\t"                \
                      INS " v[12:13], v[14:15], v[16:17]\n\t" INS " v[18:19], v[20:21], v[22:23]\n\t")     \
                 ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13",  \
                     "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23")

template <int K>
__global__ __launch_bounds__(256) void cost(int n, unsigned long long *out) {
    __shared__ double lds[1024];
    lds[threadIdx.x] = 0;
    asm volatile("v_mov_b32 v42, 0\n\t v_mov_b32 v43, 16" ::: "v42", "v43");
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
        if (K == 0) asm volatile(REP8("v_fma_f64 v[0:1], v[2:3], v[4:5], v[6:7]\n\t v_fma_f64 v[8:9], v[10:11], v[12:13], v[14:15]\n\t"
                                      "v_fma_f64 v[16:17], v[18:19], v[20:21], v[22:23]\n\t v_fma_f64 v[24:25], v[26:27], v[28:29], v[30:31]\n\t")
                                 ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31");
        if (K == 1) BODY("v_mul_f64 ");
        if (K == 2) BODY("v_add_f64 ");
        if (K == 3) asm volatile(REP8("v_mad_u64_u32 v[0:1], s[0:1], v2, v3, 0\n\t v_mad_u64_u32 v[4:5], s[2:3], v6, v7, 0\n\t"
                                      "v_mad_u64_u32 v[8:9], s[4:5], v10, v11, 0\n\t v_mad_u64_u32 v[12:13], s[6:7], v14, v15, 0\n\t")
                                 ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","s0","s1","s2","s3","s4","s5","s6","s7");
        if (K == 4) asm volatile(REP8("v_fma_f32 v0, v1, v2, v3\n\t v_fma_f32 v4, v5, v6, v7\n\t v_fma_f32 v8, v9, v10, v11\n\t v_fma_f32 v12, v13, v14, v15\n\t")
                                 ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15");
        if (K == 5) asm volatile(REP8("v_cvt_f64_f32 v[0:1], v2\n\t v_cvt_f64_f32 v[4:5], v6\n\t v_cvt_f64_f32 v[8:9], v10\n\t v_cvt_f64_f32 v[12:13], v14\n\t")
                                 ::: "v0","v1","v2","v4","v5","v6","v8","v9","v10","v12","v13","v14");
        if (K == 6) asm volatile(REP8("v_cvt_f32_f64 v0, v[2:3]\n\t v_cvt_f32_f64 v4, v[6:7]\n\t v_cvt_f32_f64 v8, v[10:11]\n\t v_cvt_f32_f64 v12, v[14:15]\n\t")
                                 ::: "v0","v2","v3","v4","v6","v7","v8","v10","v11","v12","v14","v15");
        if (K == 7) asm volatile(REP8("v_mul_u32_u24 v0, v1, v2\n\t v_mul_u32_u24 v4, v5, v6\n\t v_mul_u32_u24 v8, v9, v10\n\t v_mul_u32_u24 v12, v13, v14\n\t")
                                 ::: "v0","v1","v2","v4","v5","v6","v8","v9","v10","v12","v13","v14");
        if (K == 8) asm volatile(REP8("v_mul_hi_u32 v0, v1, v2\n\t v_mul_hi_u32 v4, v5, v6\n\t v_mul_hi_u32 v8, v9, v10\n\t v_mul_hi_u32 v12, v13, v14\n\t")
                                 ::: "v0","v1","v2","v4","v5","v6","v8","v9","v10","v12","v13","v14");
        if (K == 9) asm volatile(REP8("v_bitop3_b32 v0, v1, v2, v3 bitop3:0x96\n\t v_bitop3_b32 v4, v5, v6, v7 bitop3:0x96\n\t v_bitop3_b32 v8, v9, v10, v11 bitop3:0x96\n\t v_bitop3_b32 v12, v13, v14, v15 bitop3:0x96\n\t")
                                 ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15");
        if (K == 10) asm volatile(REP8("v_sqrt_f32 v0, v1\n\t v_sqrt_f32 v4, v5\n\t v_sqrt_f32 v8, v9\n\t v_sqrt_f32 v12, v13\n\t")
                                  ::: "v0","v1","v4","v5","v8","v9","v12","v13");
        if (K == 11) asm volatile(REP8("v_cvt_i32_f64 v0, v[2:3]\n\t v_cvt_i32_f64 v4, v[6:7]\n\t v_cvt_i32_f64 v8, v[10:11]\n\t v_cvt_i32_f64 v12, v[14:15]\n\t")
                                  ::: "v0","v2","v3","v4","v6","v7","v8","v10","v11","v12","v14","v15");
        if (K == 12) asm volatile(REP8("v_add_u32 v0, v1, v2\n\t v_add_u32 v4, v5, v6\n\t v_add_u32 v8, v9, v10\n\t v_add_u32 v12, v13, v14\n\t")
                                  ::: "v0","v1","v2","v4","v5","v6","v8","v9","v10","v12","v13","v14");
        if (K == 13) asm volatile(REP8("v_cndmask_b32 v0, v1, v2, vcc\n\t v_cndmask_b32 v4, v5, v6, vcc\n\t v_cndmask_b32 v8, v9, v10, vcc\n\t v_cndmask_b32 v12, v13, v14, vcc\n\t")
                                  ::: "v0","v1","v2","v4","v5","v6","v8","v9","v10","v12","v13","v14");
        if (K == 14) asm volatile(REP8("v_lshl_add_u64 v[0:1], v[2:3], 0, v[4:5]\n\t v_lshl_add_u64 v[6:7], v[8:9], 0, v[10:11]\n\t v_lshl_add_u64 v[12:13], v[14:15], 0, v[16:17]\n\t v_lshl_add_u64 v[18:19], v[20:21], 0, v[22:23]\n\t")
                                  ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21","v22","v23");
        if (K == 15) asm volatile(REP8("v_cndmask_b32_e64 v0, v1, v2, s[0:1]\n\t v_cndmask_b32_e64 v4, v5, v6, s[2:3]\n\t v_cndmask_b32_e64 v8, v9, v10, s[4:5]\n\t v_cndmask_b32_e64 v12, v13, v14, s[6:7]\n\t")
                                  ::: "v0","v1","v2","v4","v5","v6","v8","v9","v10","v12","v13","v14","s0","s1","s2","s3","s4","s5","s6","s7");
        if (K == 16) asm volatile(REP8("v_add_u32 v0, v1, v2\n\t v_cndmask_b32_e64 v4, v5, v6, s[2:3]\n\t v_add_u32 v8, v9, v10\n\t v_cndmask_b32_e64 v12, v13, v14, s[6:7]\n\t")
                                  ::: "v0","v1","v2","v4","v5","v6","v8","v9","v10","v12","v13","v14","s0","s1","s2","s3","s4","s5","s6","s7");
        if (K == 17) asm volatile(REP8("v_cmp_eq_u32 s[0:1], v1, v2\n\t v_cmp_eq_u32 s[2:3], v5, v6\n\t v_cmp_eq_u32 s[4:5], v9, v10\n\t v_cmp_eq_u32 s[6:7], v13, v14\n\t")
                                  ::: "v0","v1","v2","v4","v5","v6","v8","v9","v10","v12","v13","v14","s0","s1","s2","s3","s4","s5","s6","s7");
        if (K == 18) asm volatile(REP8("v_mfma_f64_16x16x4_f64 v[0:7], v[8:9], v[10:11], v[0:7]\n\t v_mfma_f64_16x16x4_f64 v[12:19], v[8:9], v[10:11], v[12:19]\n\t v_mfma_f64_16x16x4_f64 v[20:27], v[8:9], v[10:11], v[20:27]\n\t v_mfma_f64_16x16x4_f64 v[28:35], v[8:9], v[10:11], v[28:35]\n\t")
                                  ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31","v32","v33","v34","v35");
        if (K == 19) asm volatile(REP8("v_mfma_f64_16x16x4_f64 v[0:7], v[8:9], v[10:11], v[0:7]\n\t v_fma_f64 v[36:37], v[38:39], v[40:41], v[42:43]\n\t v_mfma_f64_16x16x4_f64 v[12:19], v[8:9], v[10:11], v[12:19]\n\t v_fma_f64 v[44:45], v[46:47], v[48:49], v[50:51]\n\t")
                                  ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50","v51");
        if (K == 20) asm volatile(REP8("v_mfma_f64_16x16x4_f64 v[0:7], v[8:9], v[10:11], v[0:7]\n\t v_add_u32 v36, v37, v38\n\t v_mfma_f64_16x16x4_f64 v[12:19], v[8:9], v[10:11], v[12:19]\n\t v_add_u32 v39, v40, v41\n\t")
                                  ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v36","v37","v38","v39","v40","v41");
        if (K == 21) asm volatile(REP8("v_mfma_f64_16x16x4_f64 v[0:7], v[8:9], v[10:11], v[0:7]\n\t ds_read_b128 v[36:39], v42\n\t v_mfma_f64_16x16x4_f64 v[12:19], v[8:9], v[10:11], v[12:19]\n\t ds_read_b128 v[44:47], v43\n\t")
                                  "s_waitcnt lgkmcnt(0)\n\t"
                                  ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v36","v37","v38","v39","v44","v45","v46","v47");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) atomicAdd(out, t1 - t0);
}

template <int K>
static void run(const char *name, unsigned long long *d) {
    const int n = 2000;
    (void)hipMemset(d, 0, 8);
    hipLaunchKernelGGL(cost<K>, dim3(256), dim3(256), 0, 0, n, d);
    unsigned long long h;
    (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    printf("%-18s %6.2f cycles per wave-instruction (one wave per SIMD)\n", name, h / 1024.0 / (n * 32.0));
}

int main() {
    unsigned long long *d;
    (void)hipMalloc(&d, 8);
    run<0>("warm-up", d);
    run<0>("v_fma_f64", d); run<1>("v_mul_f64", d); run<2>("v_add_f64", d); run<3>("v_mad_u64_u32", d);
    run<4>("v_fma_f32", d); run<5>("v_cvt_f64_f32", d); run<6>("v_cvt_f32_f64", d); run<7>("v_mul_u32_u24", d);
    run<8>("v_mul_hi_u32", d); run<9>("v_bitop3_b32", d); run<10>("v_sqrt_f32", d); run<11>("v_cvt_i32_f64", d);
    run<12>("v_add_u32", d); run<13>("v_cndmask_b32", d); run<14>("v_lshl_add_u64", d);
    run<15>("v_cndmask_e64 sgpr", d); run<16>("add+cndmask_e64", d); run<17>("v_cmp_eq_u32 ->s", d);
    run<18>("mfma_f64 alone", d); run<19>("mfma+fma_f64", d); run<20>("mfma+add_u32", d); run<21>("mfma+ds_read128", d);
    (void)hipFree(d);
    return 0;
}
