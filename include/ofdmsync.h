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
 *   - a pointer may be NULL when the buffer it describes is empty (B = 0 or T = 0);
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
/* packed 12-bit AXIS words, the RTL detector's wire format (ref/test_minn_preamble_detector.py:41-47,
 * ref/minn_preamble_detector.sv:152-155): per time index one word of n_ant 24-bit channel groups,
 * channel c at bit 24*c with I in its bits 0-11 and Q in 12-23 (two's complement), words packed
 * back to back little-endian (3 * n_ant bytes per time index); layout [B][T][3 * n_ant] bytes.
 * Accepted by ofs_aa_detect (OFS_FP64, 1-2 antennas) and ofs_minn_rtl (1-2 branches) on their
 * integer-exact plans; other entry points / shapes return OFS_EINVAL. */
#define OFS_CP12  3

/* arithmetic precision of a call */
#define OFS_FP32  0   /* fp32 products / in-row scans, fp64 row bases; f32/c64 outputs  */
#define OFS_FP64  1   /* fp64 throughout; f64/c128 outputs (bit-exact on integer input) */

/* status codes */
#define OFS_OK            0
#define OFS_EINVAL       -1   /* bad argument (null required pointer, bad size, bad enum)  */
#define OFS_ETOOLONG     -2   /* window/halo does not fit one workgroup's LDS tile          */
#define OFS_EHIP         -3   /* kernel launch failed (hipGetLastError)                     */
#define OFS_ESHORT       -4   /* stream shorter than one symbol (zc_freq.py:76-78 raises)   */
#define OFS_EFFT         -5   /* rocFFT plan creation / execution failed                    */

/* ofs_zc_correlate modes */
#define OFS_ZC_RAW        0   /* per-branch np.convolve(x, conj(ref[::-1]))                 */
#define OFS_ZC_V2         1   /* zc_v2 detect_zc_preamble: sum of per-branch normalised corr */
#define OFS_ZC_COMBINED   2   /* zc.py: sum_br corr / (|ref| sqrt(max(sum_br E, 0) + 1e-12)) */
#define OFS_ZC_NORMALIZE  3   /* zc_v2.normalize_correlation(corr_in, x, ref), one branch    */
#define OFS_ZC_SUM        4   /* sum_br raw corr (detect_zc_preamble, normalize=False)       */

int32_t ofs_version(void);
/* sha256 (16 hex digits) of the csrc sources (.hip, .h) and include/ofdmsync.h this library was
 * built from ("unknown" for a build without it). */
const char* ofs_source_hash(void);
const char* ofs_status_string(int32_t status);

/*
 * Debug / A-B variants (not part of the reference interface; no reference counterpart).
 * Every dispatch decision and every arithmetic choice of the library depends only on the call's
 * arguments, EXCEPT where a variant has been set through this one entry point.  Variants exist
 * so the tests can force an alternative kernel on the same input (e.g. the general LDS engine
 * against the integer-exact wave kernel, the rocFFT matched-filter pipeline against the fused LDS
 * FFT) and the measurement tools can time both.  Nothing reads the environment.  All variants
 * start unset (OFS_VARIANT_UNSET); a process that never calls ofs_debug_set_variant runs the
 * default dispatch.  Names (value meaning):
 *   EXACT        0: sync_aa / minn_rtl integer-exact and fp64 wave kernels off (general engine)
 *   FAST_E       2|4|8: samples per lane of the storing aa_fast kernel
 *   FAST_E_DO    2|4|8: samples per lane of the detect-only aa_fast kernel
 *   FAST_SCAN    32|64: row-scan precision of the storing aa_fast kernel (default 64)
 *   FAST_SCAN_DO 32|64: row-scan precision of the detect-only aa_fast kernel (default 32)
 *   RTL_WPB      1|2: streams per workgroup of rtl_exact_kernel (default 4)
 *   PARK_DIRECT  1: Park energies as direct window sums (no shared-window split)
 *   ZW64         0: zc_freq N = 4096 window FFT through zc_win_kernel instead of zc_win64_kernel
 *   ZW64_GRID    n > 0: cap of the persistent zc_win64 grid (default: CU count)
 *   ZS           0: zc_freq fp64 through the round-2 one-chunk-per-wave kernel
 *   ZF_ITEMS     n > 0: chunk-count target of that kernel (default 4096)
 *   ZS_PAIR      0: per-bin sliding DFT instead of the pair resonators
 *   ZS_DEFER     0|1: row sums per step (DPP) / deferred through LDS
 *   ZS_BPL       4: bins per lane of the one-branch sliding kernel (default 8)
 *   ZS_C         64|128|192|256: chunk length of the sliding kernels (must divide N)
 *   ZS_GBLK      0: Horner block DFTs in the pair kernel instead of Goertzel
 *   MC_FUSED     0: ZC matched filter through the rocFFT pipeline instead of the fused LDS FFT
 *   MC_FUSE_X    0: fused LDS FFT with the separate extract kernel
 *   MC_PERS      0: fused LDS FFT one block per 1024-thread workgroup instead of the persistent
 *                512-thread kernel that prefetches the next block
 *   ZC_SEQ       1: zc_v2 CFAR + gate through the sequential one-wave-per-stream kernel
 *   ZC_NODMA     1: zc_v2 CFAR tiles through registers instead of LDS-DMA
 *   BE_FAST      0: receiver back-end through the generic kernel
 *   FAST_LDS     n > 0: bytes of unused dynamic LDS per workgroup of the aa_fast kernel (occupancy
 *                cap; default 16384 for the one-antenna storing kernel = 10 per CU, 1 = no cap)
 *   OCC_LDS      n >= 0: bytes of unused dynamic LDS added to the other wave-per-stream launches
 *                (aa_stream, win_fast, aa_exact, rtl_exact, the fast back-end; occupancy A/B)
 * ofs_debug_set_variant returns OFS_EINVAL for an unknown name; value OFS_VARIANT_UNSET clears
 * one variant, ofs_debug_reset_variants clears all.  The table is per calling thread
 * (thread_local): a variant set by one thread steers only the calls that same thread makes, and
 * every new thread starts with all variants unset.  A call reads each variant once, at dispatch.
 */
#define OFS_VARIANT_UNSET INT64_MIN
int32_t ofs_debug_set_variant(const char* name, int64_t value);
int64_t ofs_debug_get_variant(const char* name);
int32_t ofs_debug_reset_variants(void);

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
 *                      L = 64*E*MR), complex64 / OFS_FP32 / 1-2 antennas / even T <= 1024;
 *   1100 + 10*E + MR : streaming wave-per-stream fast path, same arithmetic, any other T
 *                      (rows streamed from HBM, lag / window rings in registers), MR <= 8;
 *   2000 + 10*E + MR : integer-exact wave-per-stream path, OFS_CI16 / OFS_FP64, 1-2 antennas,
 *                      T * n_ant <= 2^21 (all window sums exact integers), L = 64*E*MR, MR <= 8;
 *   3000 + 10*E + MR : the same wave-per-stream kernel on OFS_C128 / OFS_FP64 input (fp64 prefix
 *                      differences over the stream, any T: the reference's running-sum error regime);
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
 * Which kernel ofs_minn_rtl dispatches a shape to (pure query): 2000 + 10*E + MW for the
 * integer-exact wave-per-stream kernel (OFS_CI16, 1-4 branches, T * n_br <= 2^21, Q = 64*E*MW
 * <= 512: metric, smoothing, threshold and gate FSM in one pass), 0 for the general engine
 * (window kernel + lane-per-stream IIR/gate kernel).
 */
int32_t ofs_rtl_plan(int32_t in_fmt, int32_t n_br, int64_t T, int32_t Q);

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
 * combined_sc_min detector front end (combined_sc_min.py:333-334: minn_streaming_metric and
 * schmidl_cox_streaming_metric on the same rx): both metrics in one pass over the input
 * (fused fp32 kernel for complex64 / 1-2 branches / N/4 a multiple of 64; otherwise the two
 * kernels above back to back).  Outputs as ofs_sc_metric (r_mode 1) and ofs_minn_metric.
 */
int32_t ofs_sc_minn_metric(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                           int32_t symbol_len, int32_t precision, void* M_sc, void* P_sc, void* R_sc,
                           void* M_minn, void* P_minn, void* R_minn, void* stream);

/*
 * Which kernel a window-metric call runs on: kind 1 = ofs_sc_metric r_mode 0, 2 = r_mode 1,
 * 3 = ofs_minn_metric, 4 = ofs_sc_minn_metric.  Returns 10*E + MW of the streaming fp32 fast kernel (win_fast.hip:
 * complex64, 1-2 branches, any T >= N, window of MW rows of 64*E samples), or 0 for the general
 * LDS-tiled engine.
 */
int32_t ofs_win_plan(int32_t kind, int32_t in_fmt, int32_t precision, int32_t n_br, int64_t T,
                     int32_t symbol_len);

/*
 * CP-correlation CFO: replaces core.estimate_cfo_from_cp (core.py:179-196), batched with a
 * per-stream CP start.  starts: [B] int64 (device); P_out: [B][2] f64 (nullable);
 * cfo_out: [B] f64.  Windows must lie inside [0, T) (checked by the caller).
 */
int32_t ofs_cp_cfo(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                   const int64_t* starts, int32_t n_fft, int32_t cp_len, double fs_hz,
                   double* P_out, double* cfo_out, void* stream);

/*
 * CP-correlation searches around an estimated CP start est[b], with
 * P_w(d) = sum_br sum_{n<win_len} x[d+n]·conj(x[d+n+n_fft]) over d in
 * [max(0, est - span), min(T - (n_fft + win_len), est + span)):
 *   mode OFS_CPS_ROBUST (0): cfo from the angle of sum_d P_w(d) — replaces
 *        core.estimate_cfo_from_cp_robust (core.py:199-231) with win_len = its `win`;
 *   mode OFS_CPS_PEAK (1):   d* = first argmax |P_w(d)|, cfo from P_w(d*) — replaces
 *        core.estimate_cfo_from_cp_peak / _peak_with_index (core.py:234-303) and
 *        core.find_cp_start_via_corr (core.py:306-336; span = search_half) with win_len = cp_len.
 * est: [B] int64; P_out [B][2] f64 and d_out [B] int64 nullable; cfo_out [B] f64;
 * status [B] int32: 0 searched, 1 empty range (the reference then falls back to
 * estimate_cfo_from_cp at est: the caller runs ofs_cp_cfo; d_out = est, cfo_out = NaN).
 * Windows are summed directly in fp64 (no prefix differences).
 */
#define OFS_CPS_ROBUST 0
#define OFS_CPS_PEAK   1
int32_t ofs_cp_search(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                      const int64_t* est, int32_t n_fft, int32_t win_len, int32_t span,
                      int32_t mode, double fs_hz, double* P_out, int64_t* d_out,
                      double* cfo_out, int32_t* status, void* stream);

/*
 * Receiver back-end after sync, batched over frames: the chain of sc.run_simulation
 * (sc.py:274-311) over core.py helpers - estimate_cfo_from_cp (core.py:179-196, skipped when
 * cfo_in is given), apply_cfo(-cfo) (:123-138) + branch mean, ofdm_fft_used (:171-176),
 * ls_channel_estimate (:339-341), estimate_timing_offset_from_phase_slope (:443-469),
 * equalize (:344-345), align_complex_gain (:357-362), evm_rms_db (:365-370).  fp64.
 *   pilot_start / data_start [B] int64: CP start of the pilot / data symbol (device);
 *   cfo_in [B] f64 or NULL; bins [n_used] int32 (device): centred subcarrier indices k, used
 *   for the gather X[k mod N] (= fftshift + (N/2 + k) % N) and as the fit's abscissa;
 *   pilot_used / data_used: c128 [.. ][n_used] known symbols, row stride (elements) per frame
 *   (0 = one row shared by all frames);  n_fft a power of two <= 4096.
 * Outputs (device, nullable): cfo_out [B], h_out / xa_out c128 [B][n_used], gain_out c128 [B],
 * evm_out, evm_db_out, slope_out (rad/bin), sto_out (samples) [B] f64.
 */
int32_t ofs_rx_backend(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                       int32_t n_fft, int32_t cp_len, double fs_hz, const int64_t* pilot_start,
                       const int64_t* data_start, const double* cfo_in, int32_t n_used,
                       const int32_t* bins, const void* pilot_used, int64_t pilot_stride,
                       const void* data_used, int64_t data_stride, double* cfo_out, void* h_out,
                       void* xa_out, void* gain_out, double* evm_out, double* evm_db_out,
                       double* slope_out, double* sto_out, void* stream);

/*
 * Batched receive-stream synthesis (benchmark / test input): the channel +
 * impairment chain of channel.apply_channel (channel.py:80-98), core.apply_cfo
 * (core.py:123-138) and sync_aa.quantize_adc (sync_aa.py:263-291):
 *   out[b][br][n] = q(base[br][off_b + n] * exp(i 2 pi cfo_b n / fs) + CN(0, 10^(-snr_b/10)))
 * with off_b ~ U{0..max_offset-1}, snr_b ~ U[snr_lo, snr_hi] dB, cfo_b ~ U[cfo_lo, cfo_hi] Hz drawn
 * per stream from Philox-4x32-10(seed, b) (distribution-level, not numpy's stream).
 *   base: [n_br][base_len] c128 (device; unit-power faded preamble, zero past its end);
 *   out_fmt OFS_C64 | OFS_C128 | OFS_CI16 (q = round(x * adc_scale) clipped to [-2048, 2047]);
 *   out: [B][n_br][T]; params: [B][3] f64 = offset, snr_db, cfo_hz (nullable).
 */
int32_t ofs_synth_batch(const void* base, int64_t base_len, int32_t n_br, int64_t B, int64_t T,
                        int32_t max_offset, double snr_lo_db, double snr_hi_db, double cfo_lo_hz,
                        double cfo_hi_hz, double fs_hz, uint64_t seed, int32_t out_fmt,
                        double adc_scale, void* out, double* params, void* stream);

/*
 * Frame synthesis: the whole per-stream chain of sync_aa.run_single_test (sync_aa.py:699-738),
 * every stream its own frame and payload:
 *   frame_b = [pre_pad zeros][preamble][n_sym random-QPSK OFDM symbols + CP][post_pad zeros]
 *             (symbols as sync_aa.build_random_qpsk_symbol, sync_aa.py:238-260: QPSK on the n_bins
 *             FFT bins `bins` (centred index k -> k mod n_fft), inverse FFT, unit power, CP);
 *   y_br     = frame_b conv cir_br (sync_aa.py:611-621); rx_br = (y_br + CN(0, mean|y_br|^2 /
 *             10^(snr_b/10))) * exp(i 2 pi cfo_b n / fs) (:622-631, :637-645);
 *   if full_scale_ratio > 0: quantize_adc(rx, rms(rx over all branches) * full_scale_ratio)
 *             (:263-291, :726-735), 12 bits;
 *   out[b][br][t] = rx_br[win_start + off_b + t] (0 outside the frame), off_b ~ U{0..max_offset-1}.
 *   preconv: [n_br][pre_len + taps - 1] c128 = preamble conv cir_br (shared part, host-built);
 *   cir: [n_br][taps] c128; n_br <= 4; n_fft a power of two <= 4096.
 *   out_fmt OFS_C64 | OFS_C128 (dequantized values if quantized) | OFS_CI16 (ADC codes when
 *   quantized); params [B][4] f64 = window start, snr_db, cfo_hz, full scale (nullable);
 *   phases [B][n_sym][n_bins] u8 = the QPSK phase indices drawn (nullable).
 */
int32_t ofs_synth_frames(const void* preconv, int64_t preconv_len, const void* cir, int64_t taps,
                         int32_t n_br, int32_t pre_pad, int32_t pre_len, int32_t n_sym, int32_t n_fft,
                         int32_t cp_len, const int32_t* bins, int32_t n_bins, int32_t post_pad, int64_t B,
                         int64_t T, int64_t win_start, int32_t max_offset, double snr_lo_db,
                         double snr_hi_db, double cfo_lo_hz, double cfo_hi_hz, double fs_hz,
                         double full_scale_ratio, uint64_t seed, int32_t out_fmt, void* out,
                         double* params, uint8_t* phases, void* stream);

/*
 * Park mirror-symmetry metric: replaces park.park_streaming_metric (park.py:64-114).
 * half = N/2; outputs for d in [half, T-half-1], n_out = T - 2*half, laid out [B][n_out]:
 *   P (c64|c128) = sum_br sum_{k<half} x[d-k]*x[d+k]; E (f32|f64) = sum_br sum_{k<half}|x[d+k]|^2;
 *   M = |P|^2 / max(E, 1e-12)^2.  Each output nullable.  T < 2*half+1 or half == 0: nothing
 *   to compute, returns OFS_OK (the reference returns empty arrays).  Tile + halo must fit
 *   LDS: N <= 8190 (fp32) / 4094 (fp64), else OFS_ETOOLONG.
 */
int32_t ofs_park_metric(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                        int32_t N, int32_t precision, void* M, void* P, void* E, void* stream);

/*
 * ZC matched filter / normaliser (fp64): replaces zc_v2.matched_filter_correlation
 * (zc_v2.py:244-254), normalize_correlation (:257-271), the branch combine of
 * detect_zc_preamble (:489-503) and the inline combiner of zc.py:106-126.
 *   ref: [N] c128 (device); ref_energy = sum |ref|^2 (host scalar, as the reference computes it);
 *   corr: c128 [B][n_br][T+N-1] (mode OFS_ZC_RAW) or [B][T+N-1] (other modes), nullable;
 *   corr_mag: f64 |corr| with the same layout, nullable (one of corr / corr_mag required);
 *   corr_in: c128 [B][T+N-1] raw correlation (OFS_ZC_NORMALIZE only, n_br must be 1).
 *   N + 2048 samples of halo must fit LDS (N <= 6100).
 */
int32_t ofs_zc_correlate(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                         const void* ref, int32_t N, double ref_energy, int32_t mode,
                         const void* corr_in, void* corr, double* corr_mag, void* stream);

/*
 * The same correlation by FFT overlap-save (SURVEY §8(f)3 "via FFT correlation"): fp64 rocFFT
 * transforms of M-sample blocks (M a power of two >= 2N, 0 = chosen to minimise the work),
 * pointwise product with FFT_M(conj(ref reversed)), inverse, then the valid outputs combined
 * and normalised per `mode` (OFS_ZC_RAW, _V2, _COMBINED, _SUM; as ofs_zc_correlate, the window
 * energy from an fp64 prefix over each block; ref_energy as ofs_zc_correlate).  The plan is made
 * for one reference (host c128, N taps) and one batch shape; `scratch` must hold *scratch_bytes (the [rows * blocks][M] c128
 * spectra), `work` *work_bytes (rocFFT work area, may be 0).  A plan carries its rocFFT execution
 * state: use it from one host thread / stream at a time (one plan per concurrent caller).
 */
int32_t ofs_zc_mf_plan_create(const void* ref, int32_t N, int64_t B, int32_t n_br, int64_t T, int32_t M,
                              void** plan_out, size_t* work_bytes, size_t* scratch_bytes);
int32_t ofs_zc_mf_plan_destroy(void* plan);
int32_t ofs_zc_correlate_fft(void* plan, int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                             double ref_energy, int32_t mode, void* corr, double* corr_mag, void* scratch,
                             void* work, void* stream);

/*
 * ZC frequency-domain metric: replaces zc_freq.compute_frequency_metric (zc_freq.py:62-99).
 * For off in [0, T-(N+cp)]: 62-bin DFT of x[off+cp : off+cp+N] at fftshift positions
 * (N/2 + bin_indices) % N, metric = |sum_br vdot(t, bins)|^2 / max(E_t * sum_br sum|bins|^2, 1e-12).
 * bin_indices [n_bins] int32 and template_bins [n_bins] c128 are HOST pointers (n_bins <= 64);
 * metric: [B][T-(N+cp)+1] (device), f64 for OFS_FP64, f32 for OFS_FP32.
 *   OFS_FP64: sliding DFT in fp64 (zc_slide.hip: block-DFT-initialised chunks, four chunks per
 *     wave; N a multiple of 64, n_br <= 2), else the one-chunk-per-wave sliding DFT (n_br <= 4).
 *   OFS_FP32: few offsets per stream (<= 64, OFS_C64, N = 64*2^j <= 4096, the cfg5 shape): a
 *     per-window 64 x N/64 pruned FFT in fp32; otherwise the fp64 sliding DFT of zc_slide.hip with
 *     the metric rounded to fp32 (n_br <= 2, N a multiple of 64, blocks within LDS), else the
 *     one-chunk-per-wave fp64 sliding DFT with the metric rounded to fp32 (n_br <= 4).
 *   n_br > 4: OFS_EINVAL (cover it, and templates of more than 64 bins, with ofs_zc_freq_partial
 *     over branch / bin groups + ofs_zc_freq_finish, as the Python mirror does).
 * Returns OFS_ESHORT when T < N + cp (the reference raises ValueError).
 */
int32_t ofs_zc_freq_metric(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                           int32_t N, int32_t cp, int32_t precision, int32_t n_bins,
                           const int32_t* bin_indices, const double* template_bins,
                           double template_energy, void* metric, void* stream);
/* which zc_freq kernel a one-branch shape runs on: 1 one-chunk-per-wave sliding DFT (fp64), 2 window
 * FFT (fp32), 3 N = 4096 window FFT with the column sums reduced across lanes (fp32; taken when the
 * template bins' residues mod 64 are distinct, as the PSS template's are, otherwise 2), 4 block-
 * initialised sliding DFT (fp64), 5 the same with the metric rounded to fp32, 6 the one-chunk-per-
 * wave sliding DFT with the metric rounded to fp32, 0 none */
int32_t ofs_zc_freq_plan(int32_t in_fmt, int32_t precision, int64_t T, int32_t N, int32_t cp);
/* Partial sums of the zc_freq metric over one group of branches and one group of template bins, so
 * any branch count and any template length reduce to kernels of <= 4 branches x <= 64 bins (the
 * reference loops over every branch and bin, zc_freq.py:85-97).  For off in [0, noff), noff =
 * T-(N+cp)+1, with bins b_{br,j} as in ofs_zc_freq_metric over branches br0 .. br0+n_grp-1 of x
 * ([B][n_br][T]) and the n_bins (<= 64) given bins:
 *   part[b][off] = (Re C, Im C, D),  C = Σ_br Σ_j conj(t_j)·b_{br,j},  D = Σ_br Σ_j |b_{br,j}|²
 * stored, or added onto part when accumulate != 0 (part: [B][noff][3] f64, device).  The groups'
 * C and D add exactly as the reference's per-branch vdot / energy sums do, before the one
 * normalisation of ofs_zc_freq_finish.  fp64 sliding DFT (one chunk of offsets per wave). */
int32_t ofs_zc_freq_partial(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T, int32_t br0,
                            int32_t n_grp, int32_t N, int32_t cp, int32_t n_bins, const int32_t* bin_indices,
                            const double* template_bins, int32_t accumulate, double* part, void* stream);
/* metric[b][off] = |C|² / max(E_t·D, 1e-12) from accumulated partial sums; f32 (OFS_FP32) or f64 out. */
int32_t ofs_zc_freq_finish(const double* part, int64_t B, int64_t noff, double template_energy,
                           int32_t precision, void* metric, void* stream);

/*
 * rocFFT leg of the ZC frequency-domain metric (zc_freq.py:62-99 and the argmax of
 * zc_freq.py:144), the north-star "rocFFT + HIP conj-mul/|.|^2/argmax" formulation, kept beside
 * the fused window-FFT kernel of ofs_zc_freq_metric for comparison (it writes and re-reads the
 * full spectrum).  A plan is a batched forward C2C rocFFT plan over n_windows = B * n_br windows
 * of N samples, input distance in_dist (= T), out-of-place into a dense [n_windows][N] spectrum;
 * it is host state owned by the caller (create once per shape, destroy when done).
 *   precision OFS_FP32: complex64 input/spectrum, f32 metric; OFS_FP64: complex128, f64 metric.
 *   work_bytes: size of the rocFFT work buffer the caller passes to ofs_zc_freq_metric_fft.
 */
int32_t ofs_zc_fft_plan_create(int32_t precision, int32_t N, int64_t n_windows, int64_t in_dist,
                               void** plan, size_t* work_bytes);
/* As ofs_zc_fft_plan_create; prune_bins > 0 (N a power of two <= 4096) makes the plan PRUNED: a
 * rocFFT store callback keeps only the template bins, so ofs_zc_freq_metric_fft's `spectrum` is
 * a compact [n_windows][prune_bins] buffer (n_bins must equal prune_bins) and the dense N-point
 * spectrum never reaches HBM.  prune_bins == 0: the dense plan. */
int32_t ofs_zc_fft_plan_create2(int32_t precision, int32_t N, int64_t n_windows, int64_t in_dist,
                                int32_t prune_bins, void** plan_out, size_t* work_bytes);
/* As ofs_zc_fft_plan_create2, executed in chunks of chunk_windows windows (0 = all n_windows in
 * one execution; a multiple of n_br at execute time): each chunk is one rocFFT execution into the
 * same [chunk][N] (or [chunk][prune_bins]) `spectrum` buffer followed by its gather, so the
 * spectrum the FFT writes is re-read from the Infinity Cache instead of HBM when chunk * N * esz
 * is well inside its 256 MiB.  ofs_zc_fft_plan_chunk returns the windows per execution (the
 * spectrum buffer's row count). */
int32_t ofs_zc_fft_plan_create3(int32_t precision, int32_t N, int64_t n_windows, int64_t in_dist,
                                int32_t prune_bins, int64_t chunk_windows, void** plan_out,
                                size_t* work_bytes);
/* ROWS plan for the reference's sliding shape (many offsets per stream): one rocFFT execution covers
 * EVERY offset of rows_per_exec consecutive [T]-sample rows (rows = stream x branch; 0 = all
 * total_rows; at execute time a multiple of n_br) - its windows start at sample cp of the first row
 * at a distance of ONE sample, (rows-1)*T + n_off of them (N a power of two <= 4096).  prune_bins =
 * n_bins: the store callback keeps the template bins of the windows that lie inside one row, spectrum
 * buffer [ofs_zc_fft_plan_chunk(plan)][prune_bins]; prune_bins = 0: no callback (rocFFT's callback
 * path blocks the host per execution), every window's dense spectrum goes to a
 * [ofs_zc_fft_plan_chunk(plan)][N] buffer and the gather reads the template bins from it.
 * ofs_zc_freq_metric_fft then issues 2 launches per row group instead of 2 per offset.  The FFTs
 * cover T instead of n_off windows per row (T / n_off times the per-offset plan's transforms). */
int32_t ofs_zc_fft_plan_create_rows(int32_t precision, int32_t N, int32_t cp, int64_t T,
                                    int64_t total_rows, int64_t rows_per_exec, int32_t prune_bins,
                                    void** plan_out, size_t* work_bytes);
int64_t ofs_zc_fft_plan_chunk(const void* plan);
int32_t ofs_zc_fft_plan_destroy(void* plan);
/*
 * For each offset off in [0, T-(N+cp)]: one batched rocFFT of x[b][br][off+cp : off+cp+N] into
 * `spectrum` ([chunk][N] device scratch, chunk = ofs_zc_fft_plan_chunk = B*n_br unless the plan
 * is chunked), then one gather kernel: metric[b][off] =
 * |sum_br vdot(t, bins)|^2 / max(E_t * sum_br sum |bins|^2, 1e-12), bins at the reference's
 * fftshift positions (N/2 + bin_indices) % N.  bin_indices [n_bins] int32, template_bins [n_bins]
 * c128: HOST pointers (n_bins <= 64).  metric [B][n_off]; peak_index [B] int64 / peak_value [B]
 * f64 (nullable) = first argmax of each row (np.argmax).  Returns OFS_ESHORT when T < N + cp.
 */
int32_t ofs_zc_freq_metric_fft(void* plan, int32_t in_fmt, const void* x, int64_t B, int32_t n_br,
                               int64_t T, int32_t N, int32_t cp, int32_t n_bins,
                               const int32_t* bin_indices, const double* template_bins,
                               double template_energy, void* spectrum, void* work, void* metric,
                               int64_t* peak_index, double* peak_value, void* stream);
/* first argmax of each row of v [B][n] (f32 | f64 per precision), np.argmax semantics (the first
 * maximal element; the first NaN if any): index [B] int64, value [B] f64, each nullable. */
int32_t ofs_row_argmax(int32_t precision, const void* v, int64_t B, int64_t n, int64_t* index,
                       double* value, void* stream);

/*
 * ZC CFAR + gate: replaces zc_v2.zc_streaming_detection (zc_v2.py:300-346) fused with
 * detect_zc_peaks (:374-446).  corr_mag: [B][n] f64.  Outputs [B][n], each nullable:
 * local_sum, corr_scaled, thresh_scaled (f64), above_threshold, metric_valid, gate_mask (u8).
 * n_events [B] int32 (total, may exceed max_events); ev_int [B][max_events][4] int64 =
 * peak_index, gate_start, gate_end, detected_start; ev_peak [B][max_events] f64 peak_value.
 * The running sum is the reference's sequential float64 recursion (bit-identical).
 */
int32_t ofs_zc_detect(const double* corr_mag, int64_t B, int64_t n, int32_t window_size,
                      int64_t thresh_value, int32_t thresh_frac_bits, double min_corr_mag,
                      int32_t reference_length, int32_t hysteresis, double* local_sum,
                      double* corr_scaled, double* thresh_scaled, uint8_t* above_threshold,
                      uint8_t* metric_valid, uint8_t* gate_mask, int32_t max_events,
                      int32_t* n_events, int64_t* ev_int, double* ev_peak, void* stream);

/* Gate alone on caller-provided flags: replaces zc_v2.detect_zc_peaks (zc_v2.py:374-446). */
int32_t ofs_zc_gate(const double* corr_mag, const uint8_t* above_threshold, const uint8_t* metric_valid,
                    int64_t B, int64_t n, int32_t reference_length, int32_t hysteresis,
                    uint8_t* gate_mask, int32_t max_events, int32_t* n_events, int64_t* ev_int,
                    double* ev_peak, void* stream);

/* ---- detection post-processing (metric streams -> timing decisions) -------------------------
 * Metrics are [B][n] device arrays; `precision` names their element type (OFS_FP32 = float,
 * OFS_FP64 = double).  Smoothed outputs are f64.  Per-stream `status` reports what the
 * reference would do: >= 0 ok (for ofs_plateau_end the branch taken), < 0 it raises ValueError.
 */

/* minn._trailing_average / combined_sc_min._trailing_average (minn.py:115-128,
 * combined_sc_min.py:167-180) of max(x, 0) when clip_negative != 0 (minn.py:149), else of x:
 * the reference's float64 running-sum recursion, sample by sample.  out: [B][n] f64. */
int32_t ofs_trailing_average(int32_t precision, const void* x, int64_t B, int64_t n, int32_t win,
                             int32_t clip_negative, double* out, void* stream);

/* sc.find_plateau_end_from_metric (sc.py:81-146).  lookahead < 0 means None.  Ms: [B][max(n, w)]
 * f64 (numpy "same" convolution length); plateau_end: [B] int64; status: [B] int32 = branch
 * (1 drop below 95 %, 2 earliest long run above 60 %, 3 slope fallback, 4 fallback on an empty
 * window, 0 empty metric), -3 where numpy's broadcast would raise. */
int32_t ofs_plateau_end(int32_t precision, const void* M, int64_t B, int64_t n, int32_t cp_len,
                        int32_t lookahead, int32_t smooth_win, double* Ms, int64_t* plateau_end,
                        int32_t* status, void* stream);

/* minn.find_minn_peak (minn.py:131-205) on the trailing average Ms (ofs_trailing_average):
 * gate = longest run of Ms >= gate_threshold * max(Ms) (earliest on ties) cut to
 * [bound_lo, bound_hi) (0, n for no bounds); empty gate -> global argmax.  peak, gate_lo,
 * gate_hi: [B] int64 (gate_* nullable); status -1 empty metric, -2 no positive peak. */
int32_t ofs_minn_peak(const double* Ms, int64_t B, int64_t n, double gate_threshold, int64_t bound_lo,
                      int64_t bound_hi, int64_t* peak, int64_t* gate_lo, int64_t* gate_hi, int32_t* status,
                      void* stream);

/* The S&C gate of combined_sc_min.run_simulation (combined_sc_min.py:337-358):
 * mask = M_sc / max >= threshold (max > 0) else M_sc >= threshold, seeded with the argmax when
 * empty.  mask: [B][n] uint8 (nullable); span: [B][2] int64 = first, last + 1 (nullable). */
int32_t ofs_sc_gate(int32_t precision, const void* M_sc, int64_t B, int64_t n, double threshold,
                    uint8_t* mask, int64_t* span, void* stream);

/* combined_sc_min._streaming_peak_detector (combined_sc_min.py:183-209) as used by
 * combined_sc_min.find_minn_peak (:212-259): first argmax (strict >) of Ms over the FIRST run of
 * mask within [bound_lo, bound_hi).  peak: [B] int64; status -1 empty gate region. */
int32_t ofs_segment_peak(const double* Ms, const uint8_t* mask, int64_t B, int64_t n, int64_t bound_lo,
                         int64_t bound_hi, int64_t* peak, int32_t* status, void* stream);


/* ------------------------------------------------------------------------------------------
 * The receiver back-end helpers one by one (the reference drivers call them individually,
 * sc.py:274-311), batched over rows, device pointers, c128 = interleaved (re, im) doubles.
 * Row operands ("ref", "den") take a row stride in elements (0 = one row shared by all).
 * ------------------------------------------------------------------------------------------ */

/* core.ofdm_fft_used (core.py:171-176): out[b][u] = fftshift(fft(x[b], n=n_fft))[(n_fft/2 +
 * bins[u]) % n_fft] = DFT_n_fft of x[b][0 : min(T, n_fft)] zero-padded, at bin bins[u] mod n_fft
 * (numpy's fft(x, n) truncates or zero-pads).  x [B][T] c64/c128/int16 I/Q; bins [n_used] int32
 * (device); out c128 [B][n_used]; n_fft a power of two <= 4096.  fp64 radix-2 FFT in LDS. */
int32_t ofs_fft_used(int32_t in_fmt, const void* x, int64_t B, int64_t T, int32_t n_fft, int32_t n_used,
                     const int32_t* bins, void* out, void* stream);

/* core.ls_channel_estimate (core.py:339-341) and core.equalize (:344-345): out = num / (den + eps)
 * with numpy's complex128 division (Smith's algorithm with the reciprocal scale, no contraction:
 * bit-identical to numpy).  num, out [B][n] c128; den [.][n] c128 with row stride den_stride. */
int32_t ofs_cdiv_eps(const void* num, int64_t B, int64_t n, const void* den, int64_t den_stride, double eps,
                     void* out, void* stream);

/* core.remove_common_phase (core.py:348-354): cpe = angle(mean(x)) when ref is NULL, else
 * angle(vdot(ref, x) / (vdot(ref, ref) + 1e-12)); out = x * exp(-i cpe).  x [B][n] c128;
 * ref [.][n] c128 (ref_stride) or NULL; cpe [B] f64; out [B][n] c128 (nullable). */
int32_t ofs_common_phase(const void* x, int64_t B, int64_t n, const void* ref, int64_t ref_stride, void* out,
                         double* cpe, void* stream);

/* core.align_complex_gain (core.py:357-362): g = vdot(x, ref) / (vdot(x, x) + eps); out = x * g.
 * gain [B] c128; out [B][n] c128 (nullable). */
int32_t ofs_align_gain(const void* x, int64_t B, int64_t n, const void* ref, int64_t ref_stride, double eps,
                       void* out, void* gain, void* stream);

/* core.evm_rms_db (core.py:365-370): evm = sqrt(mean|x - ref|^2 / mean|ref|^2),
 * evm_db = 20 log10(evm + 1e-12).  evm, evm_db [B] f64 (each nullable). */
int32_t ofs_evm(const void* x, int64_t B, int64_t n, const void* ref, int64_t ref_stride, double* evm,
                double* evm_db, void* stream);

/* core.estimate_timing_offset_from_phase_slope (core.py:443-469): phi = unwrap(angle(h)) (numpy's
 * unwrap rule), slope = Σ (k - k̄)(phi - phī) / (Σ (k - k̄)² + 1e-12) over the abscissa bins[u]
 * (centred subcarrier indices), sto = -slope * n_fft / (2 pi).  h [B][n_used] c128; slope, sto
 * [B] f64 (each nullable). */
int32_t ofs_phase_slope(const void* h, int64_t B, int32_t n_used, const int32_t* bins, int32_t n_fft,
                        double* slope, double* sto, void* stream);

/* core.apply_cfo (core.py:123-138): out[b][br][n] = x[b][br][n] * exp(i phi_n), phi_n =
 * ((2 pi cfo_b) n) * (1 / fs) - the reference's operation order (its complex scalar arithmetic
 * reduces to these two products); one tone per stream, shared by its branches.  x [B][n_br][T]
 * c64/c128/int16 I/Q; cfo_hz [B] f64 (device); out c128 [B][n_br][T]. */
int32_t ofs_apply_cfo(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T, const double* cfo_hz,
                      double fs_hz, void* out, void* stream);

/* sync_aa.quantize_adc (sync_aa.py:263-291): per component v -> round(clip(v / fs, -1, 1 - 1/L) * L)
 * / L * fs, L = 2^(bits-1), round half to even (np.round).  precision OFS_FP32: complex64 in and
 * out, every operation in fp32 (numpy 2 keeps float32 when full_scale is a Python float);
 * OFS_FP64: c64 or c128 in, c128 out (a float64 full_scale promotes).  Bit-identical to numpy. */
int32_t ofs_quantize_adc(int32_t in_fmt, const void* x, int64_t n, double full_scale, int32_t bits,
                         int32_t precision, void* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* OFDMSYNC_H */
