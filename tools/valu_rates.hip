// valu_rates.hip -- issue cost of the instruction classes the decode kernels use, on MI355X.
//
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rates.hip -o tools/valu_rates && tools/valu_rates
//
// Every wave runs a long unrolled stream of one instruction class over 8 independent register
// chains (so dependency latency is hidden); the grid puts W waves on every SIMD (W = 1, 2, 4).
// Each wave times its stream with s_memtime (shader clock cycles), so the result is the SIMD
// cycles per wave64 instruction:   elapsed cycles / (W x instructions per wave),
// independent of the clock the chip runs at.  Prints one line per (class, W).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define REP 64
#define ITERS 256

// 8 independent chains a..h; one "op" macro per class, 8 instructions per block
#define BLOCK8(OP) OP(a, b) OP(b, c) OP(c, d) OP(d, e) OP(e, f) OP(f, g) OP(g, h) OP(h, a)

template <int CLS>
__global__ void __launch_bounds__(1024) stream_kernel(uint64_t* out, uint32_t seed) {
    uint32_t a = seed + threadIdx.x, b = a * 3, c = a * 5, d = a * 7, e = a * 11, f = a * 13, g = a * 17, h = a * 19;
    double fa = a, fb = b, fc = c, fd = d, fe = e, ff = f, fg = g, fh = h;
    float sa = a, sb = b, sc = c, sd = d, se = e, sf = f, sg = g, sh = h;
    uint32_t tmp = 0;
    __syncthreads();
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int r = 0; r < REP / 8; ++r) {
            if constexpr (CLS == 0) {  // v_add_u32
#define OP(x, y) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(y));
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 1) {  // v_cndmask_b32 with an SGPR-pair mask (VOP3, as the kernels use it)
#define OP(x, y) asm volatile("v_cndmask_b32 %0, %0, %1, s[40:41]" : "+v"(x) : "v"(y));
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 2) {  // v_mov_b32_dpp row_ror (reads a chain written 7 instructions ago)
#define OP(x, y) asm volatile("v_mov_b32_dpp %0, %1 row_ror:3 row_mask:0xf bank_mask:0xf" : "+v"(x) : "v"(y));
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 3) {  // v_add_f64
#define OP(x, y) asm volatile("v_add_f64 %0, %0, %1" : "+v"(f##x) : "v"(f##y));
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 4) {  // v_fma_f64
#define OP(x, y) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(f##x) : "v"(f##y));
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 5) {  // v_min_f64 with |.| modifiers (f_minsum)
#define OP(x, y) asm volatile("v_min_f64 %0, |%0|, |%1|" : "+v"(f##x) : "v"(f##y));
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 6) {  // v_fma_f32
#define OP(x, y) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(s##x) : "v"(s##y));
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 7) {  // v_exp_f32
#define OP(x, y) asm volatile("v_exp_f32 %0, %1" : "+v"(s##x) : "v"(s##y));
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 8) {  // v_rcp_f32
#define OP(x, y) asm volatile("v_rcp_f32 %0, %1" : "+v"(s##x) : "v"(s##y));
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 9) {  // v_cvt_f32_f64
#define OP(x, y) asm volatile("v_cvt_f32_f64 %0, %1" : "+v"(s##x) : "v"(f##y));
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 10) {  // v_ldexp_f64
#define OP(x, y) asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(f##x) : "v"(y));
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 11) {  // rank rotation pair: v_sub_co_u32_dpp + v_addc_co_u32
#define OP(x, y) asm volatile("v_sub_co_u32_dpp %1, vcc, %2, %2 row_ror:5 row_mask:0xf bank_mask:0xf\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc" : "+v"(x), "=&v"(tmp) : "v"(y) : "vcc");
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 16) {  // v_add_u32 in the VOP3 (8-byte) encoding
#define OP(x, y) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(x) : "v"(y));
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 17) {  // v_add_u32 followed by s_nop 0 (counted: the VALU only)
#define OP(x, y) asm volatile("v_add_u32 %0, %0, %1\n\ts_nop 0" : "+v"(x) : "v"(y));
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 18) {  // v_add_u32 with a 32-bit literal (8 bytes)
#define OP(x, y) asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(x));
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 19) {  // v_cndmask_b32 with VCC (VOP2, 4 bytes)
#define OP(x, y) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(y));
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 20) {  // v_add_u32 followed by s_waitcnt lgkmcnt(0) (nothing outstanding)
#define OP(x, y) asm volatile("v_add_u32 %0, %0, %1\n\ts_waitcnt lgkmcnt(0)" : "+v"(x) : "v"(y));
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 21) {  // v_add_u32 followed by an independent s_add_u32 (SALU)
#define OP(x, y) asm volatile("v_add_u32 %0, %0, %1\n\ts_add_u32 s44, s44, 1" : "+v"(x) : "v"(y) : "s44", "scc");
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 12) {  // v_xor_b32 (the f/g sign work)
#define OP(x, y) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(y));
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 13) {  // v_lshrrev_b64 (64-bit shifts of the decided bits)
#define OP(x, y) asm volatile("v_lshrrev_b64 %0, %1, %0" : "+v"(f##x) : "v"(y));
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 14) {  // v_cvt_f64_f32
#define OP(x, y) asm volatile("v_cvt_f64_f32 %0, %1" : "+v"(f##x) : "v"(s##y));
                BLOCK8(OP)
#undef OP
            } else if constexpr (CLS == 15) {  // v_cmp_gt_u32 into SGPRs (ballot inputs)
#define OP(x, y) asm volatile("v_cmp_gt_u32 vcc, %0, %1" : : "v"(x), "v"(y) : "vcc");
                BLOCK8(OP)
#undef OP
            }
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    const uint32_t sink = tmp ^ a ^ b ^ c ^ d ^ e ^ f ^ g ^ h ^ (uint32_t)(fa + fb + fc + fd + fe + ff + fg + fh) ^
                          (uint32_t)(sa + sb + sc + sd + se + sf + sg + sh);
    if ((threadIdx.x & 63) == 0) {
        const int i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        out[2 * i] = (t1 - t0) | ((uint64_t)(sink & 1) << 63);
        out[2 * i + 1] = r1 - r0;  // 100 MHz reference counter
    }
}

static const char* kName[] = {"v_add_u32",     "v_cndmask_b32", "v_mov_b32_dpp", "v_add_f64",   "v_fma_f64",
                              "v_min_f64|.|",  "v_fma_f32",     "v_exp_f32",     "v_rcp_f32",   "v_cvt_f32_f64",
                              "v_ldexp_f64",   "sub_co_dpp+addc (2 instr)", "v_xor_b32", "v_lshrrev_b64",
                              "v_cvt_f64_f32", "v_cmp_gt_u32", "v_add_u32_e64 (VOP3)", "v_add_u32 + s_nop 0",
                              "v_add_u32 literal", "v_cndmask_b32 vcc (VOP2)", "v_add_u32 + s_waitcnt",
                              "v_add_u32 + s_add_u32"};

template <int CLS>
void run(uint64_t* d, uint64_t* h, int cus) {
    for (int w : {1, 2, 4}) {
        // one workgroup of 4w waves per CU: w waves on each of the 4 SIMDs
        const int waves = 4 * w, blocks = cus;
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipLaunchKernelGGL(stream_kernel<CLS>, dim3(blocks), dim3(64 * waves), 0, 0, d, 1u);
        hipDeviceSynchronize();
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(stream_kernel<CLS>, dim3(blocks), dim3(64 * waves), 0, 0, d, 2u);
        hipEventRecord(e1, 0);
        if (hipGetLastError() != hipSuccess) {
            printf("%s W=%d: launch failed\n", kName[CLS], w);
            continue;
        }
        hipDeviceSynchronize();
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(h, d, sizeof(uint64_t) * 2 * blocks * waves, hipMemcpyDeviceToHost);
        double mt = 0, rt = 0;
        for (int i = 0; i < blocks * waves; ++i) {
            mt += (double)(h[2 * i] & ~(1ULL << 63));
            rt += (double)h[2 * i + 1];
        }
        mt /= blocks * waves;
        rt /= blocks * waves;
        const double instr = (double)ITERS * REP * (CLS == 11 ? 2 : 1);
        const double ghz = mt / (rt * 10.0);  // memtime ticks per ns of the 100 MHz counter
        printf("%-26s W=%d  %6.2f cycles/instr/SIMD  (wave: %.0f memtime, %.1f us real, clock %.2f GHz; kernel %.1f us)\n",
               kName[CLS], w, mt / (w * instr), mt, rt / 100.0, ghz, ms * 1e3);
        hipEventDestroy(e0);
        hipEventDestroy(e1);
    }
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    uint64_t *d, *h = (uint64_t*)malloc(sizeof(uint64_t) * cus * 32);
    hipMalloc(&d, sizeof(uint64_t) * cus * 32);
    printf("%s, %d CUs, clock %d kHz\n", p.gcnArchName, cus, p.clockRate);
    run<0>(d, h, cus);
    run<12>(d, h, cus);
    run<1>(d, h, cus);
    run<15>(d, h, cus);
    run<2>(d, h, cus);
    run<11>(d, h, cus);
    run<13>(d, h, cus);
    run<6>(d, h, cus);
    run<7>(d, h, cus);
    run<8>(d, h, cus);
    run<3>(d, h, cus);
    run<4>(d, h, cus);
    run<5>(d, h, cus);
    run<9>(d, h, cus);
    run<14>(d, h, cus);
    run<10>(d, h, cus);
    run<16>(d, h, cus);
    run<18>(d, h, cus);
    run<19>(d, h, cus);
    run<17>(d, h, cus);
    run<20>(d, h, cus);
    run<21>(d, h, cus);
    hipFree(d);
    free(h);
    return 0;
}
