// scl_kernels.h -- parameter blocks shared by the HIP kernels and the C-ABI layer.
#ifndef PSCL_SCL_KERNELS_H
#define PSCL_SCL_KERNELS_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "polar_scl.h"

#define PSCL_MAX_WAVES_PER_WG 4

struct pscl_decode_params {
    const double* llr;  // [B][N]
    int64_t B;
    int N, n, K, L, W;
    uint64_t info_mask[2];       // bit phi set <=> phase phi is an information bit
    const uint32_t* crc_cols;    // [K] check syndrome columns (zeros when no CRC)
    const int32_t* info_set;     // [K] information positions, ascending (device)
    int has_crc;
    int sc_hard;                 // 1: successive cancellation, hard decisions (L = 1 path)
    const uint64_t* exp_table;   // [256] glibc exp table (device)
    const uint64_t* force;       // [B][2][W] or null
    int32_t* n_paths;            // [B] or null
    uint64_t* best;              // [B][W] or null
    uint8_t* flags;              // [B] or null
    double* metrics;             // [B][L] or null
    uint64_t* cands;             // [B][L][W] or null
    double* info_llrs;           // [B][L][K] or null (needs the HIST kernel)
    int rm_E;                    // NR rate matching: received length E (0 = none; llr is [B][E])
    const int32_t* rm_src;       // [N] de-interleave source index k(i) into the de-rate-matched vector
    const uint64_t* ref;         // [B][W] or null
    int k_payload;
    int64_t* counters;           // [PSCL_NCOUNT] (device)
    int fast;                    // 1: the specialised N = 128, L <= 8 kernel (scl128.hip)
    int wave_bytes;              // LDS bytes per wavefront
    int a_bytes;                 // LDS bytes of the LLR slots per wavefront
};

struct pscl_channel_params {
    uint64_t seed;
    uint32_t stream_id;
    int N, K, W, k_payload, crc_deg;
    const int32_t* info_set;     // [K] (device)
    const uint32_t* attach_cols; // [k_payload] CRC remainder columns (device)
    double sigma, noise_var;
    int64_t frame0, B;
    double* llr;                 // [B][N] (or [B][E] with rate matching)
    uint64_t* msg;               // [B][W] or null
    int rm_E;                    // NR: transmit E symbols, symbol p = x[rm_order[p % N]]
    const int32_t* rm_order;     // [N] sub-block interleaver order
};

int pscl_decode_lmax(int L);
// fills P.a_bytes / P.wave_bytes / P.fast for the kernel that will decode this shape
void pscl_decode_layout(pscl_decode_params& P, int hist);
int pscl_fast128_fstride(int L);
hipError_t pscl_launch_decode128(const pscl_decode_params& P, int hist, int wpg, int64_t grid, int lds, hipStream_t s);
int64_t pscl_decode_grid(const pscl_decode_params& P);
int pscl_decode_wpg(const pscl_decode_params& P);
int pscl_decode_lds(const pscl_decode_params& P, int hist);
hipError_t pscl_launch_decode(const pscl_decode_params& P, int hist, hipStream_t s);
hipError_t pscl_launch_channel(const pscl_channel_params& P, hipStream_t s);

#endif
