/*
 * ofdmsync.h — C ABI of the MI355X-native OFDM preamble-sync engine (libofdmsync.so).
 *
 * Drop-in boundary for the timing-metric + CFO hot path of amcolex/ofdm-sync-math.
 * The reference has no FFI: its "interface" is a set of plain Python functions
 * (SURVEY.md §8b).  Each entry point below replaces the arithmetic of one of them; the
 * Python mirror in ofdm-sync-math_amd/ (same module/function names) binds these
 * symbols with ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions (all entry points):
 *   - every pointer is a DEVICE pointer (hipMalloc'd / torch CUDA tensor storage),
 *     except where noted; buffers are caller-allocated, nothing is allocated inside;
 *   - input samples are laid out [B][n_branch][T] (stream-major, branch, time), the
 *     branch axis is SUMMED exactly like axis 0 of the reference's 2-D inputs;
 *   - outputs are laid out [B][n_out];
 *   - work is enqueued on `stream` (a hipStream_t; NULL = default stream) and is
 *     stream-ordered: no host synchronisation happens inside any call;
 *   - return value: 0 on success, negative OFS_E* on error (no partial launch on
 *     argument errors); the library keeps no global mutable state (re-entrant).
 */
#ifndef OFDMSYNC_H
#define OFDMSYNC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* input sample formats */
#define OFS_C64   0   /* interleaved float32 (re, im)                                  */
#define OFS_C128  1   /* interleaved float64 (re, im)                                  */
#define OFS_CI16  2   /* interleaved int16 (I, Q), e.g. 12-bit ADC words sign-extended  */

/* arithmetic precision of a call */
#define OFS_FP32  0   /* fp32 products / in-row scans, fp64 row bases; f32/c64 outputs  */
#define OFS_FP64  1   /* fp64 throughout; f64/c128 outputs (bit-exact on integer input) */

/* status codes */
#define OFS_OK            0
#define OFS_EINVAL       -1   /* bad argument (null required pointer, bad size, bad enum)  */
#define OFS_ETOOLONG     -2   /* window/halo does not fit one workgroup's LDS tile          */
#define OFS_EHIP         -3   /* kernel launch failed (hipGetLastError)                     */

int32_t ofs_version(void);
const char* ofs_status_string(int32_t status);

/*
 * [A][A] streaming Schmidl-Cox detector.
 * Replaces sync_aa.aa_detect_streaming (sync_aa.py:421-571): P[n], R[n], M[n], valid[n]
 * (sync_aa.py:458-493) and, if detect != 0, the gate/peak/CFO events (sync_aa.py:495-568).
 *   P: [B][T] c64|c128, R, M: [B][T] f32|f64 (per precision); valid: [B][T] uint8; each nullable
 *   (detect on a stream longer than one LDS tile needs P and M).
 *   n_events: [B] int32 (total events per stream, may exceed max_events);
 *   ev_int:  [B][max_events][4] int64 = peak_index, gate_start, gate_end, frame_start;
 *   ev_real: [B][max_events][4] f64   = P_re, P_im, M_at_peak, cfo_hz.
 */
int32_t ofs_aa_detect(int32_t in_fmt, const void* x, int64_t B, int32_t n_ant, int64_t T,
                      int32_t L, int32_t precision, void* P, void* R, void* M, uint8_t* valid,
                      int32_t detect, double threshold, int32_t hysteresis, double sample_rate,
                      int32_t max_events, int32_t* n_events, int64_t* ev_int, double* ev_real,
                      void* stream);

/*
 * Which kernel ofs_aa_detect dispatches a shape to (pure query, no launch):
 *   1000 + 10*E + MR : register-resident wave-per-stream fast path (E samples per lane,
 *                      L = 64*E*MR), complex64 / OFS_FP32 / one antenna / even T <= 1024;
 *   1                : general LDS engine, events fused (stream fits one tile);
 *   2                : general LDS engine, tiled, events in a second pass over P/M;
 *   <0               : invalid arguments or window too long (as ofs_aa_detect would return).
 */
int32_t ofs_aa_plan(int32_t in_fmt, int32_t precision, int32_t n_ant, int64_t T, int32_t L);

/*
 * Schmidl-Cox half-symbol metric, reference index convention d = 0 .. T-N.
 * r_mode 0 replaces sc.sc_streaming_metric (sc.py:42-78; R = second-half energy);
 * r_mode 1 replaces combined_sc_min.schmidl_cox_streaming_metric (combined_sc_min.py:116-164;
 * R = energy of both halves).  symbol_len = N (even).  M, P, R: [B][T-N+1], each nullable.
 */
int32_t ofs_sc_metric(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                      int32_t symbol_len, int32_t r_mode, int32_t precision,
                      void* M, void* P, void* R, void* stream);

/*
 * Minn [A A -A -A] metric: replaces minn.minn_streaming_metric (minn.py:59-112),
 * minn.minn_streaming_metric_parameterized (minn.py:697-751) and
 * combined_sc_min.minn_streaming_metric (combined_sc_min.py:60-113).  Q = symbol_len/4.
 * M, P, R: [B][T-N+1], each nullable.
 */
int32_t ofs_minn_metric(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                        int32_t symbol_len, int32_t precision, void* M, void* P, void* R,
                        void* stream);

/*
 * RTL-style adjacent-quarter Minn metric: replaces minn_rtl.minn_rtl_streaming_metric
 * (minn_rtl.py:667-733) and, if detect != 0, minn_rtl.detect_minn_rtl (minn_rtl.py:750-825).
 * Always fp64 (integer-valued inputs give the reference's exact integers).
 *   smooth_mode 0: float IIR of minn_rtl.py:706-715; 1: integer floor-shift IIR of
 *   ref/minn_preamble_detector.sv:288-296 (for integer inputs).
 *   corr_total, energy_total: [B][T] f64 (required); the other arrays nullable;
 *   n_events [B] int32; events [B][max_events][4] int64 = peak, detected, seg_start, seg_end;
 *   open_gate_start [B] int64 = start of a gate still open at the end of the stream, or -1.
 */
int32_t ofs_minn_rtl(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                     int32_t Q, int32_t smooth_shift, int32_t smooth_mode,
                     int64_t threshold_value, int32_t threshold_frac_bits,
                     double* corr_total, double* corr_positive, double* smooth_metric,
                     double* energy_total, double* corr_scaled, double* energy_scaled,
                     uint8_t* metric_valid, uint8_t* above_threshold,
                     int32_t detect, int32_t hysteresis, int32_t timing_offset,
                     int32_t max_events, int32_t* n_events, int64_t* events,
                     int64_t* open_gate_start, void* stream);

/*
 * Gate / peak FSM alone on precomputed metric arrays: replaces minn_rtl.detect_minn_rtl
 * (minn_rtl.py:750-825) when called on an existing MinnRTLMetricState.
 *   corr_positive: [B][T] f64; above_threshold, metric_valid: [B][T] uint8 (0/1);
 *   outputs as for ofs_minn_rtl.
 */
int32_t ofs_minn_rtl_gate(const double* corr_positive, const uint8_t* above_threshold,
                          const uint8_t* metric_valid, int64_t B, int64_t T,
                          int32_t hysteresis, int32_t timing_offset, int32_t max_events,
                          int32_t* n_events, int64_t* events, int64_t* open_gate_start,
                          void* stream);

/*
 * CP-correlation CFO: replaces core.estimate_cfo_from_cp (core.py:179-196), batched with a
 * per-stream CP start.  starts: [B] int64 (device); P_out: [B][2] f64 (nullable);
 * cfo_out: [B] f64.  Windows must lie inside [0, T) (checked by the caller).
 */
int32_t ofs_cp_cfo(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                   const int64_t* starts, int32_t n_fft, int32_t cp_len, double fs_hz,
                   double* P_out, double* cfo_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* OFDMSYNC_H */
