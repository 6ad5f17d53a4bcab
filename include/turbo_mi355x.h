/*
 * turbo_mi355x.h -- C ABI of the MI355X-native LTE turbo decoder (libturbo_mi355x.so).
 *
 * Plain pointers and sizes only (no HIP / torch types).  Every entry point names the
 * reference interface it replaces (/root/reference/ITTC/...).  The reference's own C++
 * entry points (TurboCodingInit / TurboEnCoding / TurboDecoding / TurboCodingRelease /
 * AWGN / Log_MAP_decoder) are provided on top of this ABI by libturbo_logmap_compat.so
 * (turbo_decoder_cuda_amd/csrc/log_map_compat.cpp), see INTEGRATION.md.
 *
 * Status codes: 0 = TD_OK; non-zero = error, message via td_last_error() (thread-local).
 * The reference has no return codes: it printf()s and exit(1)s (log_map.cpp:288-292,357-368).
 */
#ifndef TURBO_MI355X_H
#define TURBO_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TD_ABI_VERSION 1

enum td_status {
    TD_OK = 0,
    TD_EINVAL = 1,   /* bad argument (K, f1/f2, iterations, batch, null pointer) */
    TD_ENOMEM = 2,   /* host or device allocation failed */
    TD_EHIP = 3,     /* HIP runtime error (message carries hipGetErrorString) */
    TD_ENODEV = 4    /* no MI355X (gfx950) device visible */
};

/* Jacobian used by the SISO: TYPE_DECODER of ITTC/log_map.h:26-29. */
enum td_algo {
    TD_ALGO_LOGMAP = 0,  /* 16-step table max* (E_algorithm, log_map.cpp:779-801) -- the reference */
    TD_ALGO_MAXLOG = 1   /* max* = max (Max-Log-MAP, BASELINE config 3) */
};

/* Arithmetic of the decode. */
enum td_precision {
    TD_F64 = 0,   /* IEEE fp64 with the reference's operation order: the parity mode */
    TD_F32 = 1    /* fp32, same schedule and op order (throughput mode) */
};

/* Code and schedule parameters.  Reference: globals source_length/f1/f2 (ITTC/main.h:6-11,
 * main.cpp:29-37), macros N_ITERATION / TERMINATED / TYPE_DECODER (ITTC/log_map.h:24-30). */
typedef struct td_params {
    int K;            /* information bits per codeword, 1 <= K <= 10000 (MAX_FRAME_LENGTH) */
    int f1, f2;       /* QPP interleaver: pi(i) = (f1*i + f2*i*i) mod K (log_map.cpp:616-624) */
    int iterations;   /* turbo iterations (N_ITERATION) */
    int algo;         /* enum td_algo */
    int precision;    /* enum td_precision */
    int device;       /* HIP device ordinal this handle is bound to */
} td_params;

typedef struct td_handle td_handle;

/* Replaces TurboCodingInit (log_map.cpp:349-434): builds the trellis (gen_g_matrix 13/15 +
 * gen_trellis), the QPP table and the max* bucket table, on `p->device`. */
int td_create(td_handle** out, const td_params* p);
/* Replaces TurboCodingRelease (log_map.cpp:1330-1345). */
int td_destroy(td_handle* h);
/* Size the device workspace for batches up to B codewords (and, with a windowed schedule set by
 * td_set_window, the windowed schedule's buffers).  td_decode_device grows them on demand, which
 * synchronises the device; call td_reserve (after td_set_window) before a decode is captured
 * into a hipGraph. */
int td_reserve(td_handle* h, int B);
/* td_reserve of the exact schedule for B >= 1024 also picks the workspace's placement: the turbo
 * kernel's speed depends on the physical pages behind it (two modes 6-7 % apart on MI355X; the
 * slow one shows 5-8x the DRAM credit stalls), so it times one iteration on candidate workspaces
 * and keeps the fastest.  Up to TD_PLACEMENT_TRIALS candidates (environment variable, default 24;
 * 1 = a plain allocation); after at least TD_PLACEMENT_MIN candidates (default 8) the search
 * stops once one candidate runs >= 4 % below the median of those timed, never on a slow
 * straggler.  Transient memory (round 6): at most three candidates are held at a time -- the
 * slowest is released before the next one is allocated, after a 48 MiB spacer so that the next
 * does not get the same pages back -- so the search holds at most 3 workspaces + 48 MiB per probe
 * beyond the third (config 2: ~2.6 GB a workspace, <= 8.9 GB held; never more than half the free
 * device memory).  A workspace that is already big enough for B is kept as it is (placed or not):
 * call td_reserve before the first decode to have it placed.  Results do not depend on it.
 * Occupancy: a decode of more than 512 groups of 8 codewords (B > 4096 on 256 CUs) in fp32 runs
 * three or four workgroups per CU instead of two where that finishes sooner (fp32 log-MAP 1.5x,
 * Max-Log-MAP 1.6x at B = 32768); fp64 always runs two.  Bits and Le are identical either way.
 * TD_OCC3=0 (environment, read at td_create) keeps every decode on two. */

/*
 * Batched TurboDecoding (log_map.cpp:1146-1280) on device-resident data.
 *   d_llr   [B][3K+12] channel LLRs in the reference stream layout (main.cpp:202 output),
 *           double for TD_F64, float for TD_F32.  Not modified (the reference scales its
 *           buffer by 0.5 in place, :1202-1205; the compat layer reproduces that side effect).
 *   d_bits  all_iters ? [B][iterations][K] : [B][K]  uint8 hard decisions in natural order
 *           (row `it` = flow_decoded + K*it of the reference, :1261-1264).
 *   d_le    nullable, [B][iterations][2][K+3] extrinsic Le after SISO1 and SISO2
 *           (:1234-1238, :1255-1259), same dtype as d_llr.
 *   stream  hipStream_t (NULL = default stream).  Asynchronous; no host synchronisation.
 * A handle owns ONE device workspace: decodes on one handle never overlap.  A decode issued on a
 * different stream than the previous one waits on the device (hipStreamWaitEvent) until the
 * previous decode is done with the workspace; for concurrent decodes use one handle per stream.
 * A decode captured into a hipGraph (stream capture) neither waits on nor records that event, so
 * graph replays are not ordered against eager decodes on the same handle: issue them on one
 * stream, or order them with events.  Call td_reserve before capturing (no allocation inside).
 * A handle is not thread-safe: one host thread uses it at a time; handles on different threads
 * (and devices) are independent (examples/multi_gpu_decode.cpp).
 */
int td_decode_device(td_handle* h, const void* d_llr, int B, uint8_t* d_bits, int all_iters, void* d_le,
                     void* stream);

/*
 * Decoding schedule of the handle (BASELINE config 5).  NULL or window = 0
 * (the default) is the exact full-trellis schedule of log_map.cpp.  Otherwise each codeword's
 * trellis is cut into floor(L/window) sub-blocks (the last also takes the remainder, e.g. the 3
 * tail steps) decoded in parallel: a sub-block's alpha starts `overlap` steps early and its beta
 * `overlap` steps late from equal metrics, or with nii = 1 from the metrics the neighbouring
 * chain had there in the previous iteration (NII, turboDecoderBianJieZhi.cu:248,302-304,
 * 312,397-400); concurrent = 1 runs both SISOs at once on the other's extrinsic of the previous
 * iteration (turboDecoderBianJieZhi.cu:642-690) instead of the serial order; the extrinsic is
 * multiplied by ext_scale (1 = none; 0.77 in the reference GPU decoders, :423-434).  Windowed
 * decoding changes the arithmetic: its gate is the BER curve, not bit-exactness.
 *   the reference GPU decoder with P sub-blocks: {6144/P, 0, 1, 1, 0.77}, TD_ALGO_MAXLOG, TD_F32
 */
/* Debug / measurement: the windowed kernels' layout (sub-blocks per lane run of the beta kernel and
 * of the alpha kernel, batch parts on as many streams; 0 = the layout's own choice).  Results do
 * not depend on it; speed does.  Applies to the current and later td_set_window. */
int td_debug_window_layout(td_handle* h, int run, int run_a, int parts);
typedef struct td_window_params {
    int window;        /* sub-block length W (0 = exact schedule) */
    int overlap;       /* warm-up steps, 0 <= overlap <= 3*window */
    int nii;           /* 1: boundary metrics from the previous iteration */
    int concurrent;    /* 1: both SISOs concurrently (Jacobi) */
    double ext_scale;  /* extrinsic scale, (0, 4] */
} td_window_params;
/* The max* of the windowed log-MAP schedule (round 6).  TD_WMAXSTAR_FAST (the default): the
 * reference's 16-step correction (log_map.cpp:14-18, 779-801) on a finer bucket grid (8 buckets an
 * octave of d, each with the reference's value at its midpoint), read with ONE table read and no
 * threshold compare -- it differs from E_algorithm only for d within half a bucket of one of its
 * thresholds, by one table step; TD_WMAXSTAR_EXACT: E_algorithm exactly (the exact schedule's
 * form).  The windowed schedule is BER-gated either way (the BER curves of both).
 * No effect on the exact schedule or Max-Log-MAP. */
enum td_window_maxstar { TD_WMAXSTAR_FAST = 0, TD_WMAXSTAR_EXACT = 1 };
int td_set_window_maxstar(td_handle* h, int form);
/* Creates the windowed schedule's extra streams and events on the handle's device (once), so a
 * decode after td_set_window + td_reserve allocates and creates nothing and may be captured. */
int td_set_window(td_handle* h, const td_window_params* w);

/* Kernel timing (measurement support): while enabled, hipEvents on the decode stream bracket
 * the demultiplex kernel and the turbo kernel of every td_decode_device call.
 * td_profile_read synchronises on them, returns the average durations (ms) over the
 * `launches` decodes since the last read/enable, and starts a new accumulation. */
int td_profile_enable(td_handle* h, int on);
int td_profile_read(td_handle* h, float* demux_ms, float* decode_ms, int* launches);
/* Launch clock (measurement support): every exact-schedule turbo launch records, in its first
 * workgroup, the shader clock (s_memtime) and the 100 MHz real-time counter (s_memrealtime) at that
 * workgroup's start and end; a windowed decode records the same in the first workgroup of its
 * last SISO2 beta launch (round 5).  td_clock_read waits for this handle's last decode (not the
 * whole device) and returns the sustained shader clock (GHz) over that workgroup's span (ms: the
 * whole launch for the exact schedule, one workgroup's lifetime for a windowed one);
 * TD_EINVAL before any decode or when the last decode was graph-captured. */
int td_clock_read(td_handle* h, double* sclk_ghz, double* span_ms);

/* Diagnostics: in a library built with -DTD_STAMPS (td_debug_stamp_slots() > 0) the turbo
 * kernel writes per-wave shader-clock totals of its phases into d_buf [ceil(B/8)][slots]
 * (uint64).  The production library ignores the buffer and reports 0 slots. */
int td_debug_set_stamps(td_handle* h, void* d_buf);
int td_debug_stamp_slots(void);
/* Workspace placement of the last td_reserve that allocated (see td_reserve): the number of
 * candidate workspaces timed (0 = plain allocation), their probe times in ms (up to cap of them)
 * and the index kept. */
int td_debug_placement(td_handle* h, float* ms, int cap, int* pick);
/* Cost of that search: its wall time (ms) and the peak bytes of candidate workspaces it held. */
int td_debug_placement_cost(td_handle* h, double* wall_ms, double* held_bytes);
/* Bytes of the handle's decode workspace (0 before the first reserve / decode). */
int td_debug_workspace_bytes(td_handle* h, unsigned long long* bytes);
/* The placement search's stop rule on probe times ms[0..n) (host only, for tests): 1 if the search
 * would stop after them (the fast mode seen), else 0; TD_EINVAL on a bad argument. */
int td_debug_placement_rule(const float* ms, int n);

/* Trellis steps per window of the exact schedule's turbo kernel (15; fp32 at four workgroups per
 * CU runs a 12-step build).  Measurement support: bench.py's traffic model. */
int td_window_steps(void);

/* Host-pointer convenience (pageable buffers; copies, decodes, synchronises).  The device staging
 * buffers are the handle's, allocated on the first call and grown when B grows, so the per-frame
 * caller (the drop-in's TurboDecoding) allocates nothing after its first frame.
 *   out  int[B][iterations][K] exactly like the reference's flow_decoded (one row per iteration)
 *   le   nullable host [B][iterations][2][K+3]. */
int td_decode_host(td_handle* h, const void* llr, int B, int* out, void* le);

/*
 * Batched Log_MAP_decoder (log_map.cpp:898-1047) -- the SISO, host pointers.
 *   recs [B][2L] (ys, yp) pairs, La [B][L], LLR [B][L] out; dtype by h's precision.
 *   terminated: 1 = beta starts in state 0 (TERMINATED, log_map.h:24), 0 = all states equal.
 */
int td_siso_host(td_handle* h, const void* recs, const void* La, int terminated, void* LLR, int L, int B);

/*
 * Device frame generator: the frames ITTC/main.cpp makes (main.cpp:170-202)
 * -- source bits rand() % 2, TurboEnCoding, BPSK, AWGN on I and Q (mgrns, log_map.cpp:1359-1400),
 * BPSK demodulation (modanddem.cpp:189-224) -- with the process-wide glibc rand() stream of
 * srand(seed), bit-identical to the reference, generated on the GPU.
 *   td_synth_seed    srand(seed): (re)starts the handle's frame stream (main.cpp:170)
 *   td_synth_frames  the next B frames of the stream at Eb/N0 = ebn0_db:
 *                    d_info [B][K] uint8 source bits, d_llr [B][3K+12] double channel LLRs
 *                    (TurboDecoding's input).  Synchronous with respect to the host.
 */
int td_synth_seed(td_handle* h, unsigned seed);
/* Position the stream at frame `frame` of srand(seed) (each frame draws K+2 rand() values). */
int td_synth_seek(td_handle* h, unsigned long long frame);
/* Host utility behind td_synth_frames (exported for tests): the generator window
 * x[n-31 .. n-1] of srand(seed) after `draws` rand() calls; the next rand() is
 * (win[0] + win[28]) >> 1. */
int td_rand_window(unsigned seed, unsigned long long draws, uint32_t* win);
int td_synth_frames(td_handle* h, double ebn0_db, int B, uint8_t* d_info, double* d_llr, void* stream);

/* Modulation of the generator's frames (MODULATION, main.cpp:13-15, 174, 197-202): 1 = BPSK
 * (default), 2 = QPSK, 3 = 8PSK, 4 = 16QAM, 6 = 64QAM bits per symbol; SYMBOL_NUM = (3K+12)/M
 * symbols, sigma = 10^(-EbN0/20) sqrt(0.5 / (rate M)) with rate = K / SYMBOL_NUM.  TD_EINVAL when
 * 3K+12 is not a multiple of M. */
int td_synth_modulation(td_handle* h, int modulation);

/* Replaces module (modanddem.cpp:175-187, _bpsk/_qpsk/_8psk/_16qam/_64qam_module :88-173) on
 * device arrays: d_bits [nsym * modulation] uint8 (0/1; the reference takes int) -> d_si, d_sq [nsym]. */
int td_modulate(const uint8_t* d_bits, long long nsym, int modulation, double* d_si, double* d_sq, void* stream);
/* Replaces demodule (modanddem.cpp:674-685, the max-log demappers :189-671) on device arrays:
 * d_yi, d_yq [nsym] received symbols -> d_llr [nsym * modulation], bit-exact with the reference. */
int td_demodulate(const double* d_yi, const double* d_yq, long long nsym, int modulation, double Kf, double* d_llr,
                  void* stream);

/* Error counts per frame and iteration for the BER harness (main.cpp:224-237):
 * d_err[b][it] = #{i < K : d_bits[b][it][i] != d_info[b][i]}, d_bits as td_decode_device's
 * all_iters output with `iters` rows. */
int td_count_errors(td_handle* h, const uint8_t* d_bits, int iters, const uint8_t* d_info, int B, int* d_err,
                    void* stream);

/* Last error message of this thread ("" if none). */
const char* td_last_error(void);
/* Number of visible HIP devices (0 on a host without a GPU; never fails). */
int td_device_count(void);
/* ABI version of the loaded library (TD_ABI_VERSION). */
int td_abi_version(void);

/*
 * Host evaluation of the exact bucket form of E_algorithm used on the device (no GPU needed):
 * max(x,y) + table(|y-x|) through the 29-bucket LUT the kernels read from LDS.  Lets CPU
 * tests prove LUT == log_map.cpp:779-801 for every threshold.  algo = enum td_algo, or
 * TD_MAXSTAR_WINDOW_FAST: the windowed schedule's one-read table (td_set_window_maxstar).
 */
#define TD_MAXSTAR_WINDOW_FAST 2
double td_maxstar_host_f64(double x, double y, int algo);
float td_maxstar_host_f32(float x, float y, int algo);

/* Trellis tables as built by td_create's gen_trellis restatement: nextstat[8][2],
 * laststat[8][2], nextout[8][4] (ITTC/log_map.h:58-66). For tests. */
int td_trellis_tables(int* nextstat, int* laststat, int* nextout);
/* QPP permutation exactly as gen_qpp_index (log_map.cpp:616-624). For tests. */
int td_qpp_table(int K, int f1, int f2, int* pi);

#ifdef __cplusplus
}
#endif
#endif
