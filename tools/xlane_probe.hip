// xlane_probe.hip -- root-cause probe of the two cross-lane workarounds (DESIGN.md §5.2,
// §5.4): what ds_bpermute and DPP return when their source lane is inactive, and what the
// compiler makes of a DPP row_shr:1 move that feeds a subtract right after a ds_bpermute.
//
//   hipcc --offload-arch=gfx950 -O3 tools/xlane_probe.hip -o tools/xlane_probe && tools/xlane_probe
//   (hipcc ... --cuda-device-only -S tools/xlane_probe.hip: the listing shows the folded DPP form)
//
// One wavefront; every case writes its 64 lane results to global memory, the host prints them
// next to the values the "all lanes active" reading would give.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void probe(uint32_t* out, const uint32_t* perm) {
    const int lane = threadIdx.x;
    const uint32_t v = 100u + lane;
    // A: ds_bpermute inside a divergent region (lanes 0..7 active) reading lanes 8..15
    uint32_t a = 0xdeadbeef;
    if (lane < 8) a = (uint32_t)__builtin_amdgcn_ds_bpermute((lane + 8) << 2, (int)v);
    out[0 * 64 + lane] = a;
    // B: DPP row_ror:8 (bound_ctrl) inside the same divergent region
    uint32_t b = 0xdeadbeef;
    if (lane < 8) b = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, true);
    out[1 * 64 + lane] = b;
    // C: the same reads with every lane active (the reference reading)
    const uint32_t c = (uint32_t)__builtin_amdgcn_ds_bpermute(((lane & ~15) | ((lane + 8) & 15)) << 2, (int)v);
    out[2 * 64 + lane] = c;
    // D: value from lane - 1 of each 16-lane row after a ds_bpermute, left to the compiler
    // (mov_dpp row_shr:1 bound_ctrl -> may be folded into the subtract as v_sub*_dpp)
    const uint32_t w = (uint32_t)__builtin_amdgcn_ds_bpermute((int)perm[lane] << 2, (int)(v * 7u));
    const uint32_t prev = (uint32_t)__builtin_amdgcn_mov_dpp((int)w, 0x111, 0xF, 0xF, true);
    out[3 * 64 + lane] = w - prev;
    // E: the same with the move as explicit inline asm (the kernels' prev_lane32)
    uint32_t prev2;
    asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(prev2) : "v"(w));
    out[4 * 64 + lane] = w - prev2;
    out[5 * 64 + lane] = w;
    // F..I: the folded form written out, ds_bpermute + wait + NOPS + v_subrev_u32_dpp, to find
    // the wait states the LDS-return -> DPP-read sequence needs (the compiler emits s_nop 0)
    const int addr = (int)perm[lane] << 2, data = (int)(v * 7u);
    uint32_t r0, r1, r4, rc, t0, t1, t4, tc;
    asm volatile("ds_bpermute_b32 %1, %2, %3\n\ts_waitcnt lgkmcnt(0)\n\ts_nop 0\n\t"
                 "v_subrev_u32_dpp %0, %1, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                 : "=&v"(r0), "=&v"(t0) : "v"(addr), "v"(data));
    asm volatile("ds_bpermute_b32 %1, %2, %3\n\ts_waitcnt lgkmcnt(0)\n\ts_nop 1\n\t"
                 "v_subrev_u32_dpp %0, %1, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                 : "=&v"(r1), "=&v"(t1) : "v"(addr), "v"(data));
    asm volatile("ds_bpermute_b32 %1, %2, %3\n\ts_waitcnt lgkmcnt(0)\n\ts_nop 4\n\t"
                 "v_subrev_u32_dpp %0, %1, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                 : "=&v"(r4), "=&v"(t4) : "v"(addr), "v"(data));
    // I: distinct registers for the DPP source and the plain operand (copy first), s_nop 1
    asm volatile("ds_bpermute_b32 %1, %2, %3\n\ts_waitcnt lgkmcnt(0)\n\ts_nop 1\n\t"
                 "v_mov_b32 %0, %1\n\ts_nop 1\n\t"
                 "v_subrev_u32_dpp %0, %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                 : "=&v"(rc), "=&v"(tc) : "v"(addr), "v"(data));
    // J..L: distinct operands x (the DPP source) and y: which operand DPP reads, which order
    // the subtract takes.  Expected (ISA): subrev_dpp = y - x[lane-1], sub_dpp = x[lane-1] - y.
    const uint32_t x = v * 7u, y = 1000u * (uint32_t)lane;
    uint32_t rj, rk, rl;
    asm volatile("s_nop 4\n\tv_subrev_u32_dpp %0, %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                 : "=&v"(rj) : "v"(x), "v"(y));
    asm volatile("s_nop 4\n\tv_sub_u32_dpp %0, %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                 : "=&v"(rk) : "v"(x), "v"(y));
    asm volatile("s_nop 4\n\tv_subrev_u32_e32 %0, %1, %2" : "=&v"(rl) : "v"(x), "v"(y));
    out[10 * 64 + lane] = rj;
    out[11 * 64 + lane] = rk;
    out[12 * 64 + lane] = rl;
    out[13 * 64 + lane] = x;
    out[6 * 64 + lane] = r0;
    out[7 * 64 + lane] = r1;
    out[8 * 64 + lane] = r4;
    out[9 * 64 + lane] = rc;
}

int main() {
    uint32_t *d_out, *d_perm, h_perm[64], h_out[14 * 64];
    for (int i = 0; i < 64; ++i) h_perm[i] = (uint32_t)((i * 37 + 11) & 63);
    hipMalloc(&d_out, sizeof(h_out));
    hipMalloc(&d_perm, sizeof(h_perm));
    hipMemcpy(d_perm, h_perm, sizeof(h_perm), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d_out, d_perm);
    hipMemcpy(h_out, d_out, sizeof(h_out), hipMemcpyDeviceToHost);
    printf("A bpermute from inactive lanes (lanes 0-7 read 8-15):");
    for (int l = 0; l < 8; ++l) printf(" %u", h_out[l]);
    printf("\nB DPP row_ror:8 from inactive lanes (lanes 0-7):    ");
    for (int l = 0; l < 8; ++l) printf(" %u", h_out[64 + l]);
    printf("\nC same reads, all lanes active (lanes 0-7):         ");
    for (int l = 0; l < 8; ++l) printf(" %u", h_out[128 + l]);
    int bad_d = 0, bad_e = 0;
    for (int l = 0; l < 64; ++l) {
        const uint32_t w = h_out[5 * 64 + l], p = (l & 15) ? h_out[5 * 64 + l - 1] : 0u;
        bad_d += h_out[3 * 64 + l] != w - p;
        bad_e += h_out[4 * 64 + l] != w - p;
    }
    printf("\nD compiler-formed prev-lane subtract after bpermute: %d of 64 lanes wrong", bad_d);
    printf("\nE inline-asm prev-lane move:                         %d of 64 lanes wrong\n", bad_e);
    const char* nm[4] = {"F folded, s_nop 0", "G folded, s_nop 1", "H folded, s_nop 4", "I folded, copy + s_nop 1"};
    for (int c = 0; c < 4; ++c) {
        int bad = 0;
        for (int l = 0; l < 64; ++l) {
            const uint32_t w = h_out[5 * 64 + l], p = (l & 15) ? h_out[5 * 64 + l - 1] : 0u;
            bad += h_out[(6 + c) * 64 + l] != w - p;
        }
        printf("%-28s %d of 64 lanes wrong; lanes 0-3:", nm[c], bad);
        for (int l = 0; l < 4; ++l) printf(" %u", h_out[(6 + c) * 64 + l]);
        printf("  (want");
        for (int l = 0; l < 4; ++l) printf(" %u", h_out[5 * 64 + l] - (l ? h_out[5 * 64 + l - 1] : 0u));
        printf(")\n");
    }
    const char* nj[3] = {"J v_subrev_u32_dpp x,y", "K v_sub_u32_dpp x,y", "L v_subrev_u32_e32 x,y"};
    for (int c = 0; c < 3; ++c) {
        printf("%-28s lanes 1-3:", nj[c]);
        for (int l = 1; l < 4; ++l) printf(" %d", (int)h_out[(10 + c) * 64 + l]);
        printf("   y-x[l-1]:");
        for (int l = 1; l < 4; ++l) printf(" %d", (int)(1000u * l - h_out[13 * 64 + l - 1]));
        printf("  x[l-1]-y:");
        for (int l = 1; l < 4; ++l) printf(" %d", (int)(h_out[13 * 64 + l - 1] - 1000u * l));
        printf("  y-x:");
        for (int l = 1; l < 4; ++l) printf(" %d", (int)(1000u * l - h_out[13 * 64 + l]));
        printf("\n");
    }
    printf("D lanes 0-3:");
    for (int l = 0; l < 4; ++l) printf(" %u", h_out[3 * 64 + l]);
    printf("\n");
    return 0;
}
