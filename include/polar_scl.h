/*
 * polar_scl.h -- C ABI of libpolar_mi355x.so, the MI355X (gfx950) polar SC/SCL engine.
 *
 * This is the drop-in boundary for the reference's hot path (heimrih/polar_code,
 * package dl_scl_polar).  The reference has no FFI of its own: it is pure Python/NumPy,
 * so each entry point below replaces a Python function, and the binding a maintainer adds
 * on the reference side is the ctypes stub shown in INTEGRATION.md.
 *
 *   pscl_create / pscl_destroy  <- the implicit per-call setup of decode_scl
 *                                  (info mask scl.py:125-126, CRC poly crc.py:10-16)
 *   pscl_decode                 <- decode_scl(llr, info_set, M, crc, force_info_bits=...)
 *                                  dl_scl_polar/polar/scl.py:108-209, batched over B frames
 *                                  (sc_decode polar.py:130-168 is the M=1 case)
 *   pscl_decode_device          <- same, device-resident buffers, asynchronous; optionally
 *                                  folds the FER/BER counting of run_fer_sweep.py:91-109
 *   pscl_channel_device         <- the per-frame TX chain of run_fer_sweep.py:79-87
 *                                  (payload, attach_crc crc.py:19-37, encode polar.py:106-119,
 *                                  BPSK, AWGN, LLR) with a counter-based Philox stream
 *   pscl_uncoded_device         <- the uncoded BPSK baseline of run_fer_sweep.py:111-121
 *   pscl_dlscl_device           <- decode_with_retries dl_scl_polar/dlscl/flip.py:65-141 over
 *                                  a device batch (+ pscl_set_beta: the beta checkpoint)
 *   pscl_path_llrs_device       <- best_path_info_llrs / info_llrs of given paths (scl.py:158,166)
 *   pscl_simulate               <- one SNR point of run_sweep (run_fer_sweep.py:41-191): TX,
 *                                  uncoded baseline, SCL + DL-SCL, counters, in one call
 *
 * Conventions
 *   - Plain pointers and sizes only; no torch/HIP types in signatures (streams are void*).
 *   - Every function returns 0 on success or a negative PSCL_E* code; pscl_last_error()
 *     returns a thread-local message for the last failure.  The Python host layer maps
 *     PSCL_EINVAL to ValueError, PSCL_EPRUNED to RuntimeError (scl.py:171-172), the rest
 *     to RuntimeError.
 *   - Host-buffer calls are synchronous and never retain caller pointers.  Device-buffer
 *     calls are enqueued on the handle's stream (pscl_set_stream) and return immediately.
 *   - Bit vectors crossing the boundary as "words" are little-endian packed uint64:
 *     bit j of a K-bit vector is bit (j & 63) of word (j >> 6); K-bit vectors use
 *     PSCL_WORDS(K) words.
 *   - Arithmetic is IEEE fp64 end to end, like the reference (scl.py:41, polar.py:167); the
 *     path metric reproduces numpy's logaddexp (glibc exp/log1p) bit for bit.
 */
#ifndef POLAR_SCL_H
#define POLAR_SCL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSCL_ABI_VERSION 1

#define PSCL_OK 0
#define PSCL_EINVAL -1   /* bad argument (shape, range, list size, force value, CRC length) */
#define PSCL_EDEVICE -2  /* HIP runtime / device failure, or no GPU */
#define PSCL_ENOMEM -3   /* device allocation failed */
#define PSCL_EPRUNED -4  /* "All paths pruned during decoding" (cannot happen for valid input) */
#define PSCL_EUNSUP -5   /* configuration outside what the kernels implement (N, L, CRC degree) */

#define PSCL_MAX_N 1024  /* code length N: power of two, 2..1024 (N <= 128: the specialised kernels,
                            every BASELINE config; 256..1024: one wavefront per frame, global scratch;
                            the decision-LLR replay pscl_path_llrs_device stops at 128) */
#define PSCL_MAX_L 32    /* list size M/L: 1..32 (2L candidates fit one 64-lane wavefront) */
#define PSCL_MAX_CRC 32  /* CRC degree: 1..32 */
#define PSCL_WORDS(K) (((K) + 63) / 64)

/* decode flags bit layout (pscl_decode_device d_flags[b]) */
#define PSCL_FLAG_CRC_PASS 0x80u  /* best candidate passes the CRC */
#define PSCL_FLAG_IDX_MASK 0x3fu  /* index of the best candidate in the final list */

/* counters accumulated by pscl_decode_device when d_ref_words != NULL (int64[PSCL_NCOUNT]) */
#define PSCL_CNT_FRAMES 0      /* frames decoded */
#define PSCL_CNT_FRAME_ERR 1   /* best candidate fails CRC (run_fer_sweep FER, :92-94) */
#define PSCL_CNT_BIT_ERR 2     /* best bits != reference over all K bits (run_fer_sweep BER, :95-99) */
#define PSCL_CNT_PAYLOAD_ERR 3 /* frames with >=1 error in the first k_payload bits (run_ber_sweep FER) */
#define PSCL_CNT_PAYLOAD_BIT 4 /* payload bit errors (run_ber_sweep BER, :77-82) */
#define PSCL_CNT_RETRIES 5     /* flip re-decodes run by pscl_dlscl_device */
#define PSCL_NCOUNT 8

typedef struct pscl_handle pscl_handle;

/* Last error message for the calling thread ("" if none). */
const char* pscl_last_error(void);

/* ABI version compiled into the library (PSCL_ABI_VERSION). */
int pscl_abi_version(void);

/* Hash (hex) of the sources and compile flags the library was built from; the build and the
 * Python layer compare it with the sources in the tree, so a stale library is never used. */
const char* pscl_build_hash(void);

/* Number of visible HIP devices (0 when there is no GPU); negative on runtime failure. */
int pscl_device_count(void);

/*
 * Create a decoder for one polar code on one device.
 *   N        code length (power of two, 2..PSCL_MAX_N)
 *   info_set K distinct indices in [0, N), ascending (construct_info_set returns them
 *            sorted, polar.py:103); candidate bit j is u[info_set[j]] (scl.py:183).
 *            Unsorted sets are rejected with PSCL_EUNSUP.
 *   L        list size M (1..PSCL_MAX_L)
 *   crc_poly CRC generator as the integer value of the reference's hex string
 *            (e.g. 0x1864CFB for CRC-24A); 0 = no CRC (decode_scl crc=None)
 */
int pscl_create(pscl_handle** out, int device, int N, const int32_t* info_set, int K, int L,
                uint64_t crc_poly);
int pscl_destroy(pscl_handle* h);

/* Use an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL restores
 * the handle's own stream. */
int pscl_set_stream(pscl_handle* h, void* hip_stream);
void* pscl_get_stream(pscl_handle* h);
int pscl_sync(pscl_handle* h);

/*
 * Batched decode_scl on host buffers (synchronous).
 *   llr        [B][N] float64 channel LLRs (not modified)
 *   forced     NULL or [B][K] int8 in {-1,0,1}  (force_info_bits, scl.py:127-131,146-152)
 * Outputs (any may be NULL except n_paths):
 *   n_paths    [B] int32   number of paths in the final list (== min(L, 2^free_info_bits))
 *   best_bits  [B][K] int8 best_path_bits (scl.py:190-201)
 *   crc_pass   [B] uint8   check_crc(best_path_bits) (1 if crc_poly == 0)
 *   best_idx   [B] int32   index of best_path_bits in the candidate list
 *   metrics    [B][L] float64   path metrics in list order (rows >= n_paths untouched)
 *   cands      [B][L][K] int8   candidates in list order
 *   info_llrs  [B][L][K] float64 decision LLRs at info phases (scl.py:158,166)
 */
int pscl_decode(pscl_handle* h, const double* llr, int64_t B, const int8_t* forced, int32_t* n_paths,
                int8_t* best_bits, uint8_t* crc_pass, int32_t* best_idx, double* metrics, int8_t* cands,
                double* info_llrs);

/*
 * Batched sc_decode (dl_scl_polar/polar/polar.py:130-168): successive cancellation with hard
 * decisions u = (llr < 0) at information leaves, on host buffers (synchronous).
 *   bits [B][K] int8 out = u_hat[info_set]
 * The handle's list size and CRC are ignored (one path, no list, no CRC selection).
 */
int pscl_sc_decode(pscl_handle* h, const double* llr, int64_t B, int8_t* bits);

/*
 * Batched decode on device buffers, enqueued on the handle's stream.
 *   d_llr       [B][N] float64
 *   d_force     NULL or [B][2][W] uint64 (W = PSCL_WORDS(K)): force mask words, then
 *               forced-value words, indexed by info position j
 *   d_best      [B][W] uint64 best_path_bits as words (may be NULL)
 *   d_flags     [B] uint8 PSCL_FLAG_* (may be NULL)
 *   d_metrics   NULL or [B][L] float64
 *   d_cands     NULL or [B][L][W] uint64
 *   d_info_llrs NULL or [B][L][K] float64
 *   d_ref       NULL or [B][W] uint64 transmitted message words; when given, the kernel adds
 *               this batch's error statistics into d_counters (int64[PSCL_NCOUNT], device)
 *   k_payload   payload length for the PSCL_CNT_PAYLOAD_* counters (ignored if d_ref NULL)
 */
int pscl_decode_device(pscl_handle* h, const double* d_llr, int64_t B, const uint64_t* d_force,
                       uint64_t* d_best, uint8_t* d_flags, double* d_metrics, uint64_t* d_cands,
                       double* d_info_llrs, const uint64_t* d_ref, int k_payload, int64_t* d_counters);

/*
 * Generate B frames of the reference TX chain on the device (run_fer_sweep.py:79-87):
 *   payload = k_payload uniform bits; msg = attach_crc(payload) (K bits, K = k_payload + deg);
 *   u[info_set] = msg; x = polar transform(u); y = (1 - 2x) + sigma * n; llr = 2 y / sigma^2
 *   with sigma^2 = 1 / (2 * rate * 10^(ebno_db/10)).
 * Randomness: Philox4x32-10, key = (seed, stream_id), counter = (frame index, draw): frame f's
 * samples depend only on (seed, stream_id, f), so sharding frames over GPUs is exact.
 *   d_llr [B][N] float64 out;  d_msg NULL or [B][W] uint64 out (msg words)
 */
int pscl_channel_device(pscl_handle* h, uint64_t seed, uint32_t stream_id, double ebno_db, double rate,
                        int k_payload, int64_t frame0, int64_t B, double* d_llr, uint64_t* d_msg);

/*
 * Uncoded BPSK baseline (run_fer_sweep.py:111-121, --include_uncoded) counted on the device:
 * per frame k_payload payload bits (the same Philox payload block as pscl_channel_device),
 * BPSK, AWGN with sigma^2 = 1 / (2 * 10^(ebno_db/10)) (rate 1), hard decision llr < 0.
 * Noise: Philox(frame, draw 0x40000000 + pair), independent of the coded frame's noise.
 * Adds frame errors (>= 1 wrong bit) to d_counters[PSCL_CNT_FRAME_ERR], bit errors to
 * [PSCL_CNT_BIT_ERR] and B to [PSCL_CNT_FRAMES] (int64[PSCL_NCOUNT], device).
 */
int pscl_uncoded_device(pscl_handle* h, uint64_t seed, uint32_t stream_id, double ebno_db, int k_payload,
                        int64_t frame0, int64_t B, int64_t* d_counters);

/*
 * NR rate matching (dl_scl_polar/nr/polar/...): after this call the handle's decode entry
 * points take E received LLRs per frame ([B][E]) and run decode_rate_matched_scl's front end
 * (scl_nr.py:38-57) inside the decode kernel: de-rate-match (rate_match.py:19-39, repeats
 * averaged; E <= N pads with -1.0) then sub-block de-interleave (interleaver.py:26-37).
 * pscl_channel_device then transmits the interleaved, repeated codeword (scl_nr.py:23-35).
 * E = 0 switches rate matching off.  Repetition (E > N) needs N >= 32.
 */
int pscl_set_rate_match(pscl_handle* h, int E);

/*
 * Decision LLRs of given paths (scl.py:158,166 info_llrs of a path whose bits are known):
 * for frame b with information bits d_bits[b] (frozen bits 0), the leaf LLR at every
 * information phase, recomputed top-down through the same f/g operations as the decoder
 * (bit-identical to the decoder's info_llrs for that path).  Device buffers, handle stream.
 *   d_llr [B][N] (or [B][E] with rate matching);  d_bits [B][W] uint64;  d_out [B][K] float64
 */
int pscl_path_llrs_device(pscl_handle* h, const double* d_llr, int64_t B, const uint64_t* d_bits, double* d_out);

/*
 * DL-SCL flip metric matrix (dl_scl_polar/dlscl/flip.py:104-106, checkpoints/beta_M*.npy):
 * beta [K][K] row-major float64 on the host (the reference's float32 checkpoint widened
 * exactly), or NULL to rank by |L0| alone (flip.py:107).  Applies to pscl_dlscl_device.
 */
int pscl_set_beta(pscl_handle* h, const double* beta);

/*
 * SCL + DL-SCL retries over a device batch: decode_with_retries (flip.py:65-141) for every
 * frame, as run_fer_sweep.py:89-109 uses it (baseline SCL counted, then DL-SCL counted).
 * Baseline SCL decode of all B frames; the frames whose best candidate fails the CRC are
 * retried up to min(retries, K) times, each retry flipping the untried information index
 * with the smallest q = |L0| @ beta (q = |L0| without beta; ties -> lower index), forcing
 * the reference prefix, and re-decoding; the loop stops at the first CRC pass.  L0 and the
 * reference bits follow the latest attempt's best path.  Enqueued on the handle's stream;
 * the call synchronizes once (to size the retry state by the number of failing frames) and
 * returns with the retry rounds queued behind it.
 *   d_best       [B][W] uint64 out: final attempt's best bits (flip.py:126,137)
 *   d_flags      [B] uint8 out: PSCL_FLAG_* of the final attempt
 *   d_attempts   NULL or [B] int32 out: 1 + flips tried
 *   d_tried      NULL or [B][tried_stride] int32 out: flip indices in order, -1 padded
 *   d_ref        NULL or [B][W] transmitted words: baseline statistics are added into
 *                d_counters_scl, final ones into d_counters_dl (both int64[PSCL_NCOUNT],
 *                required with d_ref); PSCL_CNT_RETRIES of d_counters_dl counts re-decodes
 * Requires a CRC (without one every baseline "passes", flip.py:84-86: results = baseline).
 */
int pscl_dlscl_device(pscl_handle* h, const double* d_llr, int64_t B, int retries, uint64_t* d_best,
                      uint8_t* d_flags, int32_t* d_attempts, int32_t* d_tried, int tried_stride,
                      const uint64_t* d_ref, int k_payload, int64_t* d_counters_scl, int64_t* d_counters_dl);

/* Device scratch helpers so that non-torch callers can drive the device path. */
/*
 * One call per SNR point (the frame loop of run_fer_sweep.py:41-191 for global frames
 * [frame0, frame0 + B)): pscl_channel_device, the optional uncoded baseline
 * (pscl_uncoded_device) and SCL + DL-SCL (pscl_dlscl_device, beta from pscl_set_beta) over
 * chunks of up to 2^20 frames in handle scratch, counted on the device.  Synchronous.
 *   counters  out, host int64[3][PSCL_NCOUNT]: rows SCL, DL-SCL, uncoded (PSCL_CNT_* layout)
 * Counts depend only on (seed, stream_id, frame range): shards add up exactly.
 */
int pscl_simulate(pscl_handle* h, uint64_t seed, uint32_t stream_id, double ebno_db, double rate, int k_payload,
                  int64_t frame0, int64_t B, int retries, int include_uncoded, int64_t* counters);

/*
 * pscl_simulate without the host round trip: the point is enqueued on the handle's stream and its
 * counters ADDED into d_counters (device int64 [3][PSCL_NCOUNT]: SCL, DL-SCL, uncoded; the caller
 * zeroes them).  On a pipelined handle (pscl_set_pipelined) the point's DL-SCL retry chains
 * overlap the next call's TX and baseline decode (run_fer_sweep's next SNR point); the counters
 * are complete after pscl_join / pscl_sync / any other entry point.  Results equal pscl_simulate's.
 */
int pscl_simulate_device(pscl_handle* h, uint64_t seed, uint32_t stream_id, double ebno_db, double rate, int k_payload,
                         int64_t frame0, int64_t B, int retries, int include_uncoded, int64_t* d_counters);

int pscl_device_alloc(pscl_handle* h, void** d_ptr, int64_t bytes);
/* (pscl_device_free first orders and completes the handle's pending pipelined work, which may
 * still use the buffer) */
int pscl_device_free(pscl_handle* h, void* d_ptr);
int pscl_memcpy_htod(pscl_handle* h, void* d_dst, const void* src, int64_t bytes);
int pscl_memcpy_dtoh(pscl_handle* h, void* dst, const void* d_src, int64_t bytes);
int pscl_memset_device(pscl_handle* h, void* d_dst, int value, int64_t bytes);

/*
 * Screening decode (default on).  Plain decodes (no metrics, candidates, decision LLRs, path
 * counts, forced bits) of the compiled-in N = 128 codes and of the long codes (N = 256..1024 at
 * L = 4, 8) run a screening pass whose path metrics carry a tail log1p(exp(-|v|)) with a
 * measured absolute error bound (fp32 exp2/log2; the bound checked exhaustively over every fp32
 * input on the device); every list ordering it decides must clear a margin of twice the N-term
 * metric error bound, and frames where one does not are re-decoded by the exact kernel.  Decoded
 * bits, CRC flags and best indices are identical to the exact decode (decode_scl,
 * dl_scl_polar/polar/scl.py:108-209).  enable = 0 runs the exact kernel only.
 */
int pscl_set_screening(pscl_handle* h, int enable);

/* Frames the last screening decode on this handle handed to the exact re-decode (synchronizes
 * the stream; 0 if no screening decode ran).  Diagnostic / test hook. */
int pscl_screening_count(pscl_handle* h, int64_t* count);

/*
 * Pipelined plain decodes (throughput mode; the reference's run_sweep frame loop,
 * run_fer_sweep.py:41-191, over a stream of independent batches).  With enable = 1 a plain
 * pscl_decode_device that takes the screening path leaves its exact re-decode of the deferred
 * frames on a second stream, where it overlaps the caller's next decode: when the call returns,
 * that re-decode is not yet ordered into the handle's stream.  Its input rows, output rows and
 * counters stay in use until pscl_join, pscl_sync, any other entry point on the handle (each
 * orders the pending re-decodes into the handle's stream first) or the second following
 * pipelined decode.  Consecutive pipelined decodes must not write the same output buffers.
 * pscl_dlscl_device (one chunk) likewise: a pipelined call enqueues its baseline decode, then the
 * previous pipelined call's retry rounds and DL counters (on high-priority streams, beside this
 * call's baseline), and leaves its own rounds to the next call or the join.  The retry chains of
 * consecutive calls alternate two stream sets, so they run beside each other.  enable = d in
 * 2..4 deepens the DL-SCL pipeline: a pscl_dlscl_device call's input, output and counter buffers
 * are free again at the d-th following pipelined call (enable = 1: the second), so a caller
 * cycling d output buffers lets the chains of up to d - 1 calls run behind the baselines.
 * Results are bit-identical to the non-pipelined form.  enable = 0 (default) restores
 * stream-ordered completion.  Timing (pscl_timing_*) of a pipelined decode covers its
 * screening launch only.  PSCL_EINVAL for enable outside 0..4.
 */
int pscl_set_pipelined(pscl_handle* h, int enable);
/* Order the pending pipelined re-decodes into the handle's stream (no host wait on the plain
 * decodes' re-decodes; a pending pipelined DL-SCL call's chains are enqueued here, which waits for
 * that call's baseline decode on the host to read its failing-frame count). */
int pscl_join(pscl_handle* h);

/*
 * Tuning and test knobs of one handle (value 0 restores the default, which is the measured best
 * schedule).  The library reads no environment variables: a knob changes only
 * the handle it is set on, never a result (every schedule is bit-identical).  Pending pipelined
 * work is ordered first.  PSCL_EINVAL for an unknown knob or a value out of range.
 *   PSCL_TUNE_DL_SCREEN     DL-SCL retry decodes on the forced-bit screening instance (where the
 *                           code has one): 1 always, 2 never, 0 (default) every retry chain, or
 *                           with PSCL_TUNE_DL_SCREEN_MIN set the chains it selects
 *   PSCL_TUNE_DL_CHUNKS     1..64: baseline chunks of a DL-SCL call (default 1)
 *   PSCL_TUNE_DL_SPLIT      1..2: retry chains per chunk (default 2; 1 when pipelined)
 *   PSCL_TUNE_SIDE_PRIORITY 1: a pipelined handle's side streams at normal priority (default high)
 *   PSCL_TUNE_POST_GRID     16..4096: workgroup cap of the DL-SCL post pass (default 512)
 *   PSCL_TUNE_RETRY_WPG     1..4: wavefronts per workgroup of the retry decodes (default: by LDS)
 *   PSCL_TUNE_DL_SCREEN_MIN 1..2^30: with PSCL_TUNE_DL_SCREEN = 0, screen only the retry chains of
 *                           at least this many entries and those beside a later baseline decode (a
 *                           pipelined call's or a chunk's); 0 (default): no threshold
 *   PSCL_TUNE_DL_LANE       1: a DL-SCL baseline decode (N = 128) on the lane-per-path screening
 *                           kernel (default); 2: on the two-lanes-per-path one
 *   PSCL_TUNE_DL_RETRY_LANE 2: screened retry decodes (N = 128) on the two-lanes-per-path forced-
 *                           bit instance instead of the lane-per-path one (default)
 *   PSCL_TUNE_DL_STREAMS    0..3 (bit mask): 1 the side chain on its main chain's stream, 2 one chain
 *                           set (consecutive calls' chains on the same streams, in call order)
 *   PSCL_TUNE_POST_PAIRS    1..32: entry pairs per wavefront the DL-SCL post pass grid is sized for
 *                           (default 2, PSCL_POST_PAIRS in dlscl.hip; capped by PSCL_TUNE_POST_GRID)
 *   PSCL_TUNE_TX_FUSED      pscl_simulate[_device] of the (128,64) code at L = 4, 8: 1 the baseline
 *                           decode draws its channel rows itself (the TX chain fused into the lane
 *                           kernel: no channel_kernel launch, no LLR rows written but those of
 *                           failing or deferred frames), 2 the separate TX launch; 0 (default):
 *                           the measured faster of the two
 *   PSCL_TUNE_DL_FUSED_POST 1: a screened retry round of the (128,64) code at L = 4, 8 runs its post
 *                           pass in the decode kernel (one launch per round; warm-start metrics
 *                           from the screening tail, deferred entries exact from phase 0); 2: the
 *                           separate dl_post_kernel; 0 (default): the measured faster
 *   PSCL_TUNE_POST_EPW      2 or 4: entries a wavefront of the DL-SCL post pass works on at once in
 *                           its narrow form (pipelined calls; 32 or 16 lanes per entry); 0 (default):
 *                           the measured faster
 *   PSCL_TUNE_LANE_EXACT    exact decodes of the (128,64) and NR (128,88) codes at L = 4, 8 -- the
 *                           deferred frames' re-decode and the exact DL-SCL retry rounds: 1 on the
 *                           exact lane-per-path kernel, 2 on the two-lanes-per-path exact kernel;
 *                           3 (tests) also every plain decode, unscreened; 0 (default): the measured
 *                           faster
 *   PSCL_TUNE_DL_WARM_APX   1: the screened DL-SCL chain's warm-start metrics from the screening tail
 *                           (the post pass skips the exact tails; entries its decodes defer start
 *                           the side chain's exact decode at phase 0), 2: exact warm-start metrics;
 *                           0 (default): the measured faster
 *   PSCL_TUNE_DL_TAIL       1: a pipelined DL-SCL call's baseline tail (the re-decode of its deferred
 *                           frames, the compaction of the failing ones) on the handle's stream, before
 *                           the next call's baseline; 0 (default): on a stream of its own beside it
 */
#define PSCL_TUNE_DL_SCREEN 1
#define PSCL_TUNE_DL_CHUNKS 2
#define PSCL_TUNE_DL_SPLIT 3
#define PSCL_TUNE_SIDE_PRIORITY 4
#define PSCL_TUNE_POST_GRID 5
#define PSCL_TUNE_RETRY_WPG 6
#define PSCL_TUNE_DL_LANE 7
#define PSCL_TUNE_DL_SCREEN_MIN 8
#define PSCL_TUNE_DL_RETRY_LANE 9
#define PSCL_TUNE_POST_PAIRS 10
#define PSCL_TUNE_DL_STREAMS 11
#define PSCL_TUNE_TX_FUSED 12
#define PSCL_TUNE_DL_FUSED_POST 13
#define PSCL_TUNE_POST_EPW 14
#define PSCL_TUNE_LANE_EXACT 15
#define PSCL_TUNE_DL_WARM_APX 16
#define PSCL_TUNE_DL_TAIL 17
#define PSCL_TUNE_COUNT 18
int pscl_set_tuning(pscl_handle* h, int knob, int64_t value);

/*
 * Diagnostic: the metric tail log1p(exp(-|v|)) (scl.py:102-105) of n device values, evaluated
 * as the decode kernels do -- d_exact by the bit-exact glibc port, d_apx by the screening
 * decode's bounded-error form.  Device buffers, handle stream.
 */
int pscl_softplus_tails_device(pscl_handle* h, const double* d_v, int64_t n, double* d_exact, double* d_apx);

/*
 * Diagnostic (the screening margin's proof obligation): the absolute error of the screening
 * metric tail against the bit-exact glibc port for every fp32 bit pattern x32 in [lo, hi].
 * d_out[2] (device, zeroed by the caller): d_out[0] = fp64 bits of the largest error, d_out[1]
 * = (its high word << 32) | the x32 bit pattern of the largest error.  Handle stream.
 */
int pscl_tail_abs_scan_device(pscl_handle* h, uint32_t lo, uint32_t hi, uint64_t* d_out);

/*
 * The same scan for the bits form of the screening tail (the lane kernels' plain decodes):
 * max |pscl_tail2_f32(y32) - log1p(exp(-y32 ln 2)) / ln 2| over the fp32 bit patterns [lo, hi],
 * the reference being the bit-exact glibc port in fp64 (glibc_softplus.h).  Same output layout.
 */
int pscl_tail2_scan_device(pscl_handle* h, uint32_t lo, uint32_t hi, uint64_t* d_out);

/*
 * Kernel timing with HIP events recorded on the launch stream around every decode kernel
 * launch (enable = 1 starts a fresh accumulation).  pscl_timing_read returns the number of
 * timed launches and their summed duration in milliseconds (synchronizes the stream).
 */
int pscl_timing_enable(pscl_handle* h, int enable);
int pscl_timing_read(pscl_handle* h, int64_t* launches, double* total_ms);
/* The same, split by stream: launches on the handle's stream (a plain decode's screening pass,
 * a DL-SCL call's baseline decode) and on its side streams (DL-SCL retry decodes).  Side-stream
 * launches overlap main-stream ones, so the two sums are not additive in wall time.  Any output
 * pointer may be NULL. */
int pscl_timing_read_split(pscl_handle* h, int64_t* main_launches, double* main_ms, int64_t* side_launches,
                           double* side_ms);

/*
 * Host-side cost of the DL-SCL calls (pscl_dlscl_device, also through pscl_simulate[_device]):
 * the calls' summed wall time on the host, the part of it spent blocked in the one host wait a
 * call may make (its previous pipelined call's failing-frame count, a finished baseline decode),
 * and the number of calls -- so busy (enqueue) time = call_ms - wait_ms.  reset = 1 zeroes the
 * accumulators after reading.  Any output pointer may be NULL.
 */
int pscl_host_stats(pscl_handle* h, double* call_ms, double* wait_ms, int64_t* calls, int reset);

/*
 * Which schedules this handle has enqueued since it was created (tests assert the path they
 * mean to exercise ran): DL-SCL retry rounds whose post pass ran inside the screened retry
 * decode (PSCL_TUNE_DL_FUSED_POST), rounds with the separate dl_post_kernel, and pscl_simulate
 * blocks whose TX was fused into the baseline decode (PSCL_TUNE_TX_FUSED), dl_post_kernel
 * launches in the 4-entries-per-wavefront form (PSCL_TUNE_POST_EPW), and exact decodes launched on
 * the exact lane-per-path kernel (PSCL_TUNE_LANE_EXACT).  Any pointer may be NULL.
 */
int pscl_path_stats(pscl_handle* h, int64_t* fused_post_rounds, int64_t* post_rounds, int64_t* fused_tx_blocks,
                    int64_t* post_epw4_launches, int64_t* lane_exact_launches);

/*
 * The product's host (CPU) decoder: pscl_decode's contract and outputs (bit-identical) without a
 * GPU or a handle -- decode_scl (dl_scl_polar/polar/scl.py:108-209) for the reference's
 * CPU-only runs (BASELINE config 1: run_fer_sweep on CPU).  Any power-of-two N <= PSCL_MAX_N,
 * 1 <= L <= 255, crc_poly as pscl_create (0 = none); forced as pscl_decode ({-1, 0, 1} per info
 * bit, or NULL); bits, cands as int8 0/1.  Frames are split over `threads` host threads (0 = all
 * hardware threads).  PSCL_EINVAL for invalid arguments.  No HIP call is made.
 */
int pscl_decode_cpu(int N, const int32_t* info_set, int K, int L, uint64_t crc_poly, const double* llr, int64_t B,
                    const int8_t* forced, int32_t* n_paths, int8_t* best_bits, uint8_t* crc_pass, int32_t* best_idx,
                    double* metrics, int8_t* cands, double* info_llrs, int threads);

/* Launch geometry used by the decode kernel (for roofline bookkeeping): waves per
 * workgroup, workgroups per launch for B frames, LDS bytes per workgroup. */
int pscl_launch_info(pscl_handle* h, int64_t B, int* waves_per_wg, int64_t* grid, int* lds_bytes);

#ifdef __cplusplus
}
#endif

#endif /* POLAR_SCL_H */
