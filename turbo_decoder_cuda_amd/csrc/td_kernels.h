// td_kernels.h -- launch interface between the C ABI (td_api.cpp) and td_kernels.hip.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

#include "td_tables.h"

namespace td {

// Per-lane trellis constants of the rotating-label scheme (td_kernels.hip header), indexed
// [phase = step mod 3][slot = lane & 7]; built and verified on the host (build_lane_tables).
struct LaneTables {
    int state[3][8];                     // state held by slot l at a step of phase ph
    // gamma of a transition = sg * G with G = P (sel 0) or Q (sel 1), sg = +1 (u = 1) / -1 (u = 0),
    // P = (ys + yp) + La/2, Q = (ys - yp) + La/2 (see td_kernels.hip, "gamma")
    int a_sg[3][8], a_sel[3][8];         // alpha step, self transition
    int a_pg[3][8], a_psel[3][8];        // alpha step, partner transition
    int b_sg[3][8], b_sel[3][8];         // beta step, self transition
    int b_pg[3][8], b_psel[3][8];        // beta step, partner transition
    int a_j[3][8];                       // state produced by the alpha step of phase ph
    int a_swap[3][8];                    // 1 if the self transition has input u = 1
};

// Builds the tables from the trellis; false if the code is not the 8-state shift-register
// butterfly the labeling assumes (never for 13/15).
bool build_lane_tables(const Trellis& t, LaneTables& lt);

// Kernel parameter block (passed by value).  Device arrays are batch-interleaved:
// group g = codewords 8g..8g+7, element [g][step][c].
constexpr int kPermPad = 32;         // spare ints after pi / pinv: the loader stages window-sized chunks
constexpr int kGroupWaves = 4;       // waves per codeword group (stamp slots per group)
constexpr int kCuSlotKeys = 2048;    // (XCC, SE, SH, CU) keys of HW_ID
// Trellis steps per window of the exact schedule (td_kernels.hip kW): a multiple of 3 (the label
// period) with at most 128 (step, codeword) fold items (two fold waves, one item per lane), so 12 or
// 15.  The library builds 15 (td_kernels.hip) and 12 (td_kernels_w12.hip, fp32 at four per CU); the
// host sizes every buffer for the larger and reads the decode's own window count from
// td::window_steps().
constexpr int kWindowStepsMax = 15;
// Alpha scratch (astore): group-major [G][L+1][64] (8 codewords x 8 states per step and group; row L
// holds log-MAP's alpha_raw[.][L], whose max is beta's first tempmax), plus two windows of the longest
// window length after the last group: the loader copies whole windows (and the first rows of the
// window after the last), so the last group's copies read past its rows.  (Window-major and
// step-major layouts and pads between the groups' streams were measured in round 3: none removed the
// placement modes of DESIGN.md 3.2, and group-major had the fastest fast mode.)
constexpr size_t astore_group_elems(int L) { return ((size_t)L + 1) * 64; }
constexpr size_t astore_elems(int G, int L) { return (size_t)G * astore_group_elems(L) + (size_t)2 * kWindowStepsMax * 64; }

template <typename T>
struct DecodeParams {
    T* sys1;   // [G][L][8] systematic of decoder 1 (x0.5)
    T* par1;   // [G][L][8] parity 1
    T* sys2;   // [G][L][8] interleaved systematic (decoder 2)
    T* par2;   // [G][L][8] parity 2
    T* ext12;  // [G][K][8] Le of decoder 1 scattered to interleaved order (= La of decoder 2)
    T* ext21;  // [G][K][8] Le of decoder 2 scattered to natural order (= La of decoder 1)
    T* astore;    // F pass -> B pass scratch by 8c + state, [G][L+1][64] (astore_elems): log-MAP alpha_raw of
                  // rows 0..L; Max-Log-MAP the normalised alpha of the rows i = 0 mod 3
    T* tmstore;   // [G][L][8] tempmax[i+1] per step and codeword: Max-Log-MAP only (log-MAP forms it from
                  // the alpha_raw rows on chip; its workspace carries no tmstore region)
    T* llr_out;                 // bare SISO: [G][L][8]
    const int* pi;              // [K] QPP
    const int* pinv;            // [K] inverse QPP
    const LutEntry<T>* lut;     // [kLutSize]
    const T* qlut;              // [kQRows] the windowed schedule's one-read max* table (build_qlut)
    uint8_t* bits;              // decisions (see td_decode_device)
    T* le_dump;                 // nullable
    unsigned long long* stamps; // diagnostic build (TD_STAMPS) only: [G][6] phase cycle totals
    unsigned long long* clk;    // nullable: workgroup 0's (shader clock, 100 MHz real time) at its start and
                                // end, [4] (td_clock_read: the launch's sustained shader clock)
    int K, L, nT, G, B, iters, all_iters, algo;
    int role_cus;               // CU count for the second-round role rotation (wg_pos); 0 = off
    int occ3;                   // 1: large batches on three workgroups per CU where built (turbo_decode_kernel3)
    int sys2_in_turbo;          // 1: the turbo kernel forms sys2 = sys1 o pi itself (first SISO's F pass),
                                // launch_demux skips demux_perm_kernel (exact schedule only)
    unsigned* cu_slots;         // [kCuSlotKeys] per-CU occupancy bits (placement-based roles, wg_pos)
    int nextstat[kStates][2];
    int laststat[kStates][2];
    int nextout[kStates][4];
    const LaneTables* lane;     // device copy (dynamic per-lane indexing stays out of scratch)
};

// demultiplex + x0.5 of the stream into the batch-interleaved arrays
template <typename T>
hipError_t launch_demux(const DecodeParams<T>& p, const T* flow, hipStream_t st);
// the same into the windowed schedule's wide arrays [B/64][L][64] (sys2 included)
template <typename T>
hipError_t launch_window_demux(const DecodeParams<T>& p, const T* flow, hipStream_t st);
// the turbo iterations (one wave per 8 codewords)
template <typename T>
hipError_t launch_turbo(const DecodeParams<T>& p, hipStream_t st, bool probe = false);   // probe: td_reserve's placement probe symbol
// fp32 at four workgroups per CU, from td_kernels_w12.hip (td_kernels.hip built with 12-step windows,
// whose fp32 LDS fits four per CU; the default 15-step windows fit three)
template <typename T, int ALGO>
hipError_t launch_turbo4_w12(const DecodeParams<T>& p, hipStream_t st);

// sliding-window mode (BASELINE config 5, td_set_window): sub-blocks of `window` steps
struct WindowParams {
    int window;        // sub-block length W (the last sub-block also takes L mod W)
    int overlap;       // warm-up steps g
    int nii;           // boundary metrics from the previous iteration
    int concurrent;    // both SISOs per launch on the previous iteration's extrinsics
    double ext_scale;  // extrinsic scaling (1 = none)
    int run;           // sub-blocks per lane run, 0 = chosen by window_run (td_debug_window_layout)
    int run_a;         // the alpha kernel's, if non-zero (td_debug_window_layout)
    int parts;         // batch parts on as many streams, 0 = 2 (td_debug_window_layout)
    int exact_table;   // 1: log-MAP with log_map.cpp's E_algorithm exactly (three-read bucket table);
                       // 0: the one-read table of build_qlut (td_set_window_maxstar)
};
// extra device buffers of the windowed schedule
template <typename T>
struct WindowBufs {
    T* ext12[2];   // [B/64][K][64] x2 (concurrent schedule: iteration parity); serial uses [0]
    T* ext21[2];
    T* nii;        // [2 parity][2 dec][B][nS][2][8]
    T* ckpt[2];    // per decoder alpha checkpoints (window_ckpt_elems; serial: one shared)
    uint8_t* bitsT;  // [K][Bp] SISO2's decisions before bits_transpose_kernel (window_bits_bytes)
};
// sub-blocks per codeword (the last also takes L mod W) and the checkpoint scratch per decoder
inline int window_subblocks(int L, int W) { return L / W > 0 ? L / W : 1; }
size_t window_ckpt_elems(int B, int L, int W, bool f32);
size_t window_bits_bytes(int B, int K);
// sub-blocks per lane run of the windowed kernels (1 = one sub-block per lane); `force` > 0 asks for
// that many where runs are possible (g <= W, W a multiple of the checkpoint spacing S)
int window_run(int L, int W, int g, int B, int ndec, int S, int force = 0);
// the handle's second stream and its fork / join events (timing disabled); st2 null: one stream
// the windowed schedule's batch parts run on the caller's stream (part 0) and st[1..] (launch_window_algo)
constexpr int kSwMaxParts = 4;
struct WindowStreams {
    hipStream_t st[kSwMaxParts];   // st[0] unused
    hipEvent_t fork[kSwMaxParts], join[kSwMaxParts];
};
template <typename T>
hipError_t launch_window(const DecodeParams<T>& p, const WindowParams& w, const WindowBufs<T>& wb, hipStream_t st,
                         const WindowStreams& ws);

template <typename T>
hipError_t launch_siso(const DecodeParams<T>& p, const T* recs, const T* la, T* la_ws, int terminated, T* llr,
                       hipStream_t st);

// device frame generator (td_synth.hip): main.cpp's frame, one thread per frame
struct SynthParams {
    int K, n, B;
    int M;                  // bits per symbol (MODULATION): 1, 2, 3, 4, 6
    const int* pi;          // [K] QPP
    const uint32_t* win;    // [B][31] glibc random_r window at each frame's first draw
    double sigma, Kf;       // main.cpp:174 sigma; demodule's 1/(2 sigma^2), computed on the host
    uint8_t* info;          // [B][K] source bits out
    double* flow;           // [B][3K+12] channel LLRs out (fp64, the reference's type)
};
hipError_t launch_synth(const SynthParams& p, hipStream_t st);
// module / demodule (modanddem.cpp:175, :674) on device arrays
hipError_t launch_modulate(const uint8_t* bits, long long nsym, int M, double* si, double* sq, hipStream_t st);
hipError_t launch_demodulate(const double* yi, const double* yq, long long nsym, int M, double Kf, double* out,
                             hipStream_t st);
hipError_t launch_count_errors(const uint8_t* bits, const uint8_t* info, int K, int iters, int B, int* err,
                               hipStream_t st);

int window_steps();   // steps per window of the exact schedule's two-per-CU kernel (td_kernels.hip kW)

}  // namespace td
