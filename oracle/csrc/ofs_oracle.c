/*
 * ofs_oracle.c — C restatement of the reference's [A][A] streaming detector.
 *
 * TEST / BASELINE INFRASTRUCTURE ONLY: used by tests/ as a second checker and by bench.py's
 * cpu_baseline leg as the timed CPU port ("kind": "port").  Never linked into the product.
 *
 * Statement-for-statement restatement of sync_aa.aa_detect_streaming (sync_aa.py:421-571):
 * per antenna a DelayLine(L) (:368-386), a complex RunningSum(L) of x[n]·conj(x[n-L])
 * (:321-342) and a real RunningSum(L) of |x[n]|² (:345-365), all updated once per sample
 * with the reference's recursion  sum = sum + sample - oldest;  then the metric (:486-493)
 * and the gate / peak / CFO state machine (:495-568).  Streams are independent: OpenMP
 * parallelises over streams only.
 *
 * Parity: pinned in tests/test_oracle_c.py against the reference's golden vectors.
 */
#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif
#include <complex.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
    double complex* dl;   /* delay line ring, L entries */
    double complex* pr;   /* complex running-sum ring */
    double* rr;           /* real running-sum ring */
    double complex psum;
    double rsum;
    int64_t ptr, dfill, pfill, rfill;
} ant_state;

static void detect_one(const void* xv, int is_c128, int64_t na, int64_t T, int64_t L,
                       double thr, int hyst, double fs, double* P, double* R, double* M,
                       int max_ev, int32_t* n_ev_out, int64_t* ev_i, double* ev_r,
                       double* scratch_m, double* scratch_p) {
    ant_state* st = (ant_state*)calloc((size_t)na, sizeof(ant_state));
    for (int64_t a = 0; a < na; ++a) {
        st[a].dl = (double complex*)calloc((size_t)L, sizeof(double complex));
        st[a].pr = (double complex*)calloc((size_t)L, sizeof(double complex));
        st[a].rr = (double*)calloc((size_t)L, sizeof(double));
    }
    double* Mloc = scratch_m;           /* M[n]                          */
    double* Ploc = scratch_p;           /* P[n] re/im interleaved        */
    unsigned char* valid = (unsigned char*)malloc((size_t)(T > 0 ? T : 1));
    for (int64_t n = 0; n < T; ++n) {
        double complex P_sum = 0.0;
        double R_sum = 0.0;
        int all_valid = 1;
        for (int64_t a = 0; a < na; ++a) {
            ant_state* s = &st[a];
            double complex x;
            if (is_c128) {
                const double* p = (const double*)xv + 2 * (a * T + n);
                x = p[0] + I * p[1];
            } else {
                const float* p = (const float*)xv + 2 * (a * T + n);
                x = (double)p[0] + I * (double)p[1];
            }
            /* DelayLine.step (sync_aa.py:377-386) */
            const int64_t k = s->ptr;
            double complex xd = s->dl[k];
            s->dl[k] = x;
            int dvalid = 1;
            if (s->dfill < L) { s->dfill++; xd = 0.0; dvalid = 0; }
            /* product (sync_aa.py:469) */
            const double complex prod = dvalid ? x * conj(xd) : 0.0;
            /* RunningSum.step (sync_aa.py:331-342) */
            const double complex oldp = s->pr[k];
            s->pr[k] = prod;
            s->psum = s->psum + prod - oldp;
            int pvalid = 1;
            if (s->pfill < L) { s->pfill++; pvalid = 0; }
            /* RunningSumReal.step on |x|^2 (sync_aa.py:355-365, :475-477) */
            const double h = hypot(creal(x), cimag(x));
            const double pw = h * h;
            const double oldr = s->rr[k];
            s->rr[k] = pw;
            s->rsum = s->rsum + pw - oldr;
            int rvalid = 1;
            if (s->rfill < L) { s->rfill++; rvalid = 0; }
            s->ptr = (k + 1 == L) ? 0 : k + 1;
            P_sum += s->psum;
            R_sum += s->rsum;
            all_valid = all_valid && pvalid && rvalid;
        }
        double m = 0.0;
        if (all_valid && R_sum > 1e-6 * (double)L) {
            const double ap = hypot(creal(P_sum), cimag(P_sum));
            m = (ap * ap) / (R_sum * R_sum);
            if (m > 1.0) m = 1.0;
        }
        Mloc[n] = m;
        Ploc[2 * n] = creal(P_sum);
        Ploc[2 * n + 1] = cimag(P_sum);
        valid[n] = (unsigned char)all_valid;
        if (P) { P[2 * n] = creal(P_sum); P[2 * n + 1] = cimag(P_sum); }
        if (R) R[n] = R_sum;
        if (M) M[n] = m;
    }
    /* gate / peak / CFO (sync_aa.py:495-568) */
    int gate_open = 0, n_ev = 0;
    int64_t gate_start = 0, peak_index = 0, low_count = 0;
    double pk_re = 0.0, pk_im = 0.0, peak_mag = 0.0;
    for (int64_t n = 0; n < T; ++n) {
        if (!valid[n]) continue;
        const double m = Mloc[n];
        const double ap = hypot(Ploc[2 * n], Ploc[2 * n + 1]);
        const double pm = ap * ap;
        if (!gate_open) {
            if (m >= thr) {
                gate_open = 1; gate_start = n; peak_index = n;
                pk_re = Ploc[2 * n]; pk_im = Ploc[2 * n + 1]; peak_mag = pm; low_count = 0;
            }
        } else {
            if (pm > peak_mag) { peak_index = n; pk_re = Ploc[2 * n]; pk_im = Ploc[2 * n + 1]; peak_mag = pm; }
            if (m >= thr) {
                low_count = 0;
            } else {
                low_count += 1;
                if (low_count >= hyst) {
                    if (n_ev < max_ev) {
                        int64_t* e = ev_i + 4 * n_ev;
                        double* r = ev_r + 4 * n_ev;
                        e[0] = peak_index; e[1] = gate_start; e[2] = n; e[3] = peak_index - 2 * L + 1;
                        r[0] = pk_re; r[1] = pk_im; r[2] = Mloc[peak_index];
                        r[3] = atan2(pk_im, pk_re) * fs / (2.0 * M_PI * (double)L);
                    }
                    n_ev++;
                    gate_open = 0; peak_mag = 0.0; low_count = 0;
                }
            }
        }
    }
    if (gate_open) {
        if (n_ev < max_ev) {
            int64_t* e = ev_i + 4 * n_ev;
            double* r = ev_r + 4 * n_ev;
            e[0] = peak_index; e[1] = gate_start; e[2] = T; e[3] = peak_index - 2 * L + 1;
            r[0] = pk_re; r[1] = pk_im; r[2] = Mloc[peak_index];
            r[3] = atan2(pk_im, pk_re) * fs / (2.0 * M_PI * (double)L);
        }
        n_ev++;
    }
    *n_ev_out = n_ev;
    for (int64_t a = 0; a < na; ++a) { free(st[a].dl); free(st[a].pr); free(st[a].rr); }
    free(st);
    free(valid);
}

/* x: [B][na][T] complex (c64 if is_c128 == 0, else c128), host memory.
 * P: [B][T][2] f64, R/M: [B][T] f64 (each nullable); n_ev [B]; ev_i [B][max_ev][4];
 * ev_r [B][max_ev][4].  nthreads <= 0: OpenMP default. */
int oracle_aa_detect(const void* x, int is_c128, int64_t B, int64_t na, int64_t T, int64_t L,
                     double thr, int hyst, double fs, double* P, double* R, double* M,
                     int max_ev, int32_t* n_ev, int64_t* ev_i, double* ev_r, int nthreads) {
    if (!x || B < 0 || na < 1 || T < 0 || L < 1 || max_ev < 0 || !n_ev) return -1;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    int rc = 0;
#pragma omp parallel
    {
        double* sm = (double*)malloc(sizeof(double) * (size_t)(T > 0 ? T : 1));
        double* sp = (double*)malloc(sizeof(double) * 2 * (size_t)(T > 0 ? T : 1));
        if (!sm || !sp) {
#pragma omp atomic write
            rc = -2;
        }
#pragma omp for schedule(dynamic, 16)
        for (int64_t b = 0; b < B; ++b) {
            if (!sm || !sp) continue;
            const size_t esz = is_c128 ? 16 : 8;
            const void* xb = (const char*)x + (size_t)b * (size_t)na * (size_t)T * esz;
            detect_one(xb, is_c128, na, T, L, thr, hyst, fs, P ? P + 2 * b * T : NULL,
                       R ? R + b * T : NULL, M ? M + b * T : NULL, max_ev, n_ev + b,
                       ev_i + 4 * (int64_t)max_ev * b, ev_r + 4 * (int64_t)max_ev * b, sm, sp);
        }
        free(sm);
        free(sp);
    }
    return rc;
}

/* ------------------------------------------------------------------------------------------
 * minn_rtl: statement-for-statement restatement of minn_rtl._DelayLine (minn_rtl.py:512-542),
 * _RunningSum (:545-580), _antenna_path (:583-652), minn_rtl_streaming_metric (:667-733, float
 * smoothing) and detect_minn_rtl (:750-825).  x: [B][nb][T] complex128 (re, im interleaved).
 * Outputs (each [B][T], nullable): corr_total, corr_positive, smooth, energy_total, corr_scaled,
 * energy_scaled (f64), metric_valid, above (u8); events [B][max_ev][4] int64 = (peak_index,
 * detected_index, seg_start, seg_end); n_ev [B]; open_start [B] (-1: none).
 * ------------------------------------------------------------------------------------------ */
typedef struct { double* mem; int64_t depth, wr, fill; double last; } rtl_delay;
typedef struct { double* mem; int64_t depth, wr, fill; double sum; int valid; } rtl_rsum;

static double rtl_delay_step(rtl_delay* d, double v, int in_valid, int* out_valid) {
    if (d->depth == 0) { if (in_valid) d->last = v; *out_valid = in_valid; return v; }
    if (!in_valid) { *out_valid = 0; return d->last; }
    const double rd = d->fill < d->depth ? 0.0 : d->mem[d->wr];
    d->mem[d->wr] = v;
    d->wr = (d->wr + 1) % d->depth;
    if (d->fill < d->depth) { d->fill++; d->last = 0.0; *out_valid = 0; return 0.0; }
    d->last = rd; *out_valid = 1; return rd;
}

static double rtl_rsum_step(rtl_rsum* r, double v, int in_valid, int* out_valid) {
    if (r->depth == 0) { if (in_valid) { r->sum = v; r->valid = 1; } *out_valid = r->valid; return r->sum; }
    if (!in_valid) { *out_valid = r->valid; return r->sum; }
    const double oldest = r->fill < r->depth ? 0.0 : r->mem[r->wr];
    r->mem[r->wr] = v;
    r->wr = (r->wr + 1) % r->depth;
    r->sum = r->sum + v - oldest;
    if (r->fill < r->depth) { r->fill++; if (r->fill >= r->depth) r->valid = 1; } else r->valid = 1;
    *out_valid = r->valid;
    return r->sum;
}

static void rtl_one(const double* x, int64_t nb, int64_t T, int64_t Q, int shift, int64_t thr, int frac,
                    int hyst, int toff, int max_ev, double* ct, double* cpos, double* sm, double* et,
                    double* cs, double* es, unsigned char* mv, unsigned char* ab, int64_t* ev, int32_t* n_ev,
                    int64_t* open_start, double* w_ct, double* w_et, unsigned char* w_v, double* w_cp,
                    unsigned char* w_ab) {
    for (int64_t n = 0; n < T; ++n) { w_ct[n] = 0.0; w_et[n] = 0.0; w_v[n] = 1; }
    double* buf = (double*)calloc((size_t)(7 * (Q > 0 ? Q : 1)), sizeof(double));
    for (int64_t br = 0; br < nb; ++br) {
        const double* xs = x + 2 * br * T;
        rtl_delay di = {buf, Q, 0, 0, 0.0}, dq = {buf + Q, Q, 0, 0, 0.0};
        rtl_rsum cw = {buf + 2 * Q, Q, 0, 0, 0.0, 0}, ew = {buf + 3 * Q, Q, 0, 0, 0.0, 0};
        rtl_delay cd = {buf + 4 * Q, Q, 0, 0, 0.0}, e1 = {buf + 5 * Q, Q, 0, 0, 0.0}, e2 = {buf + 6 * Q, Q, 0, 0, 0.0};
        memset(buf, 0, sizeof(double) * (size_t)(7 * Q));
        double cr = 0.0, cp = 0.0, er = 0.0, ep = 0.0, ep2 = 0.0;
        for (int64_t n = 0; n < T; ++n) {
            const double in_i = xs[2 * n], in_q = xs[2 * n + 1];
            int v0, v1, cv, ev_, cpv, eqv, e2v;
            const double d_i = rtl_delay_step(&di, in_i, 1, &v0);
            const double d_q = rtl_delay_step(&dq, in_q, 1, &v1);
            const double qp = d_i * in_i + d_q * in_q;                       /* minn_rtl.py:616 */
            const double pw = in_i * in_i + in_q * in_q;                     /* :617 */
            const double csum = rtl_rsum_step(&cw, qp, 1, &cv);
            const double esum = rtl_rsum_step(&ew, pw, 1, &ev_);
            const double cpv_ = rtl_delay_step(&cd, csum, cv, &cpv);
            const double eq = rtl_delay_step(&e1, esum, ev_, &eqv);
            const double e2q = rtl_delay_step(&e2, eq, eqv, &e2v);
            if (cv) cr = csum;
            if (cpv) cp = cpv_;
            if (ev_) er = esum;
            if (eqv) ep = eq;
            if (e2v) ep2 = e2q;
            w_ct[n] += cr + cp;                                               /* :695-702 */
            w_et[n] += er + ep + ep2;
            w_v[n] = w_v[n] && e2v;
        }
    }
    free(buf);
    double s = 0.0;
    const double denom = (double)(1LL << (shift > 0 ? shift : 0));
    for (int64_t n = 0; n < T; ++n) {
        const double c = w_ct[n] > 0.0 ? w_ct[n] : 0.0;                      /* :704 */
        if (w_v[n]) s = (shift == 0) ? c : s + (c - s) / denom;              /* :709-715 */
        const double c_s = s * (double)(1LL << frac);
        const double e_s = thr == 0 ? 0.0 : w_et[n] * (double)thr;           /* :718-721 */
        const int a = w_v[n] && (c_s >= e_s);
        w_cp[n] = c; w_ab[n] = (unsigned char)a;
        if (ct) ct[n] = w_ct[n];
        if (cpos) cpos[n] = c;
        if (sm) sm[n] = s;
        if (et) et[n] = w_et[n];
        if (cs) cs[n] = c_s;
        if (es) es[n] = e_s;
        if (mv) mv[n] = w_v[n];
        if (ab) ab[n] = (unsigned char)a;
    }
    /* detect_minn_rtl (minn_rtl.py:750-825) */
    int gate_open = 0, k = 0;
    int64_t gs = -1, pk = 0, low = 0;
    double pv = 0.0;
    const int64_t limit = hyst > 0 ? hyst - 1 : 0;
    for (int64_t n = 0; n < T; ++n) {
        if (!w_v[n]) continue;
        const double m = w_cp[n];
        if (!gate_open) {
            if (w_ab[n]) { gate_open = 1; gs = n; pv = m; pk = n; low = 0; }
        } else {
            if (m >= pv) { pv = m; pk = n; }
            if (w_ab[n]) {
                low = 0;
            } else {
                int closing = 0;
                if (hyst == 0) closing = 1;
                else if (low == limit) closing = 1;
                else low++;
                if (closing) {
                    if (k < max_ev) {
                        int64_t* e = ev + 4 * k;
                        e[0] = pk; e[1] = pk + toff; e[2] = gs >= 0 ? gs : n; e[3] = n + 1;
                    }
                    k++;
                    gate_open = 0; gs = -1; pv = 0.0; low = 0;
                }
            }
        }
    }
    *n_ev = k;
    *open_start = (gate_open && gs >= 0) ? gs : -1;
}

int oracle_minn_rtl(const double* x, int64_t B, int64_t nb, int64_t T, int64_t Q, int shift, int64_t thr,
                    int frac, int hyst, int toff, int max_ev, double* ct, double* cpos, double* sm, double* et,
                    double* cs, double* es, unsigned char* mv, unsigned char* ab, int64_t* ev, int32_t* n_ev,
                    int64_t* open_start, int nthreads) {
    if (!x || B < 0 || nb < 1 || T < 0 || Q < 1 || max_ev < 0 || !n_ev || !open_start) return -1;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    int rc = 0;
#pragma omp parallel
    {
        const size_t t1 = (size_t)(T > 0 ? T : 1);
        double* w_ct = (double*)malloc(sizeof(double) * t1);
        double* w_et = (double*)malloc(sizeof(double) * t1);
        double* w_cp = (double*)malloc(sizeof(double) * t1);
        unsigned char* w_v = (unsigned char*)malloc(t1);
        unsigned char* w_ab = (unsigned char*)malloc(t1);
        if (!w_ct || !w_et || !w_cp || !w_v || !w_ab) {
#pragma omp atomic write
            rc = -2;
        }
#pragma omp for schedule(dynamic, 16)
        for (int64_t b = 0; b < B; ++b) {
            if (!w_ct || !w_et || !w_cp || !w_v || !w_ab) continue;
            const int64_t o = b * T;
#define RTL_P(p) ((p) ? (p) + o : NULL)
            rtl_one(x + 2 * b * nb * T, nb, T, Q, shift, thr, frac, hyst, toff, max_ev, RTL_P(ct), RTL_P(cpos),
                    RTL_P(sm), RTL_P(et), RTL_P(cs), RTL_P(es), RTL_P(mv), RTL_P(ab), ev + 4 * (int64_t)max_ev * b,
                    n_ev + b, open_start + b, w_ct, w_et, w_v, w_cp, w_ab);
#undef RTL_P
        }
        free(w_ct); free(w_et); free(w_cp); free(w_v); free(w_ab);
    }
    return rc;
}

int oracle_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ------------------------------------------------------------------------------------------
 * Full-batch checkers of the fp32 fast paths (cfg4, cfg5): the reference's fp64 values are
 * recomputed here per stream and the engine's fp32 outputs compared against them under a stated
 * error model, without materialising fp64 copies of multi-GB outputs.  Per-stream statistics
 * out; the tests assert on them.  Error-model constants come from the caller (the test states
 * and justifies them).
 * ------------------------------------------------------------------------------------------ */
typedef long double ld;

static inline void ld_cjmul(const double* x, const double* y, ld* re, ld* im) {
    /* x · conj(y) */
    *re = (ld)x[0] * y[0] + (ld)x[1] * y[1];
    *im = (ld)x[1] * y[0] - (ld)x[0] * y[1];
}

/* combined_sc_min.schmidl_cox_streaming_metric (combined_sc_min.py:116-164): half = N/2,
 *   P(d) = Σ_br Σ_{k<half} x[d+k]·conj(x[d+half+k]), R(d) = Σ_br Σ_{k<N} |x[d+k]|²,
 *   M = |P|² / max(R, 1e-12)²;
 * combined_sc_min.minn_streaming_metric (:60-113, = minn.py:59-112): Q = N/4,
 *   P(d) = Σ_br [Σ_{k<Q} q0·conj(q1) + Σ_{k<Q} q2·conj(q3)], R(d) = Σ_br Σ |q1|²+|q2|²+|q3|²,
 *   M = max(Re P, 0)² / max(R, 1e-12)²;   d in [0, T - N].
 * The window sums are long-double prefix differences (64-bit mantissa: below 1e-18 of a window's
 * absolute sum for these lengths) - the reference's direct sums to far below fp32 resolution.
 * Alongside each P, S = Σ |x[i]|·|x[i+lag]| over the same terms (the absolute sum of the error
 * model).  Output o[8][n_out]: Pc re, Pc im, Rc, Sc, Pm re, Pm im, Rm, Sm. */
static void scm_ref_one(const double* x, int64_t nb, int64_t T, int64_t N, ld* pre, double* o) {
    const int64_t half = N / 2, Q = N / 4, nout = T - N + 1;
    ld* aH = pre;                 /* prefix of x[i]·conj(x[i+half]) (re, im), |.|, lag half  */
    ld* aQ = pre + 3 * (T + 1);   /* prefix of x[i]·conj(x[i+Q]) (re, im), |.|, lag Q        */
    ld* eP = pre + 6 * (T + 1);   /* prefix of |x[i]|²                                        */
    for (int64_t d = 0; d < 8 * nout; ++d) o[d] = 0.0;
    for (int64_t br = 0; br < nb; ++br) {
        const double* xs = x + 2 * br * T;
        ld sh[3] = {0, 0, 0}, sq[3] = {0, 0, 0}, se = 0;
        for (int64_t i = 0; i <= T; ++i) {
            aH[3 * i] = sh[0]; aH[3 * i + 1] = sh[1]; aH[3 * i + 2] = sh[2];
            aQ[3 * i] = sq[0]; aQ[3 * i + 1] = sq[1]; aQ[3 * i + 2] = sq[2];
            eP[i] = se;
            if (i == T) break;
            const double* xi = xs + 2 * i;
            se += (ld)xi[0] * xi[0] + (ld)xi[1] * xi[1];
            const ld ax = sqrtl((ld)xi[0] * xi[0] + (ld)xi[1] * xi[1]);
            if (i + half < T) {
                ld r, m;
                const double* y = xs + 2 * (i + half);
                ld_cjmul(xi, y, &r, &m);
                sh[0] += r; sh[1] += m; sh[2] += ax * sqrtl((ld)y[0] * y[0] + (ld)y[1] * y[1]);
            }
            if (i + Q < T) {
                ld r, m;
                const double* y = xs + 2 * (i + Q);
                ld_cjmul(xi, y, &r, &m);
                sq[0] += r; sq[1] += m; sq[2] += ax * sqrtl((ld)y[0] * y[0] + (ld)y[1] * y[1]);
            }
        }
        for (int64_t d = 0; d < nout; ++d) {
            double* od = o;
            od[0 * nout + d] += (double)(aH[3 * (d + half)] - aH[3 * d]);
            od[1 * nout + d] += (double)(aH[3 * (d + half) + 1] - aH[3 * d + 1]);
            od[2 * nout + d] += (double)(eP[d + N] - eP[d]);
            od[3 * nout + d] += (double)(aH[3 * (d + half) + 2] - aH[3 * d + 2]);
            const int64_t a0 = d, a1 = d + Q, a2 = d + 2 * Q, a3 = d + 3 * Q;
            od[4 * nout + d] += (double)((aQ[3 * a1] - aQ[3 * a0]) + (aQ[3 * a3] - aQ[3 * a2]));
            od[5 * nout + d] += (double)((aQ[3 * a1 + 1] - aQ[3 * a0 + 1]) + (aQ[3 * a3 + 1] - aQ[3 * a2 + 1]));
            od[6 * nout + d] += (double)(eP[d + N] - eP[d + Q]);
            od[7 * nout + d] += (double)((aQ[3 * a1 + 2] - aQ[3 * a0 + 2]) + (aQ[3 * a3 + 2] - aQ[3 * a2 + 2]));
        }
    }
}

/* Error model of one window metric (u = 2^-24, the fp32 unit roundoff), oracle values P, R, S:
 *   |ΔP| <= kP·u·S + u·|P|      |ΔR| <= kR·u·R
 *   |ΔM| <= 2·(c/R)·(bP/R) + (bP/R)² + 2·M·(bR/R) + kM·u·M       (c = |P| or max(Re P, 0))
 * i.e. first-order propagation of the P and R errors through M = c²/R² plus the metric's own
 * fp32 operations. */
static inline double fp32_metric_bound(double c, double R, double M, double bP, double bR, double kM) {
    const double Rm = R > 1e-12 ? R : 1e-12;
    const double p = bP / Rm;
    return 2.0 * (c / Rm) * p + p * p + 2.0 * M * (bR / Rm) + kM * 0x1p-24 * M + 1e-300;
}

/* x: [B][nb][T] complex (c64 or c128).  Engine outputs [B][T-N+1]: Mc, Pc (c64), Rc (combined
 * S&C) and Mm, Pm, Rm (Minn), fp32.  stats [B][8]:
 *   0 max|ΔMc|   1 max |ΔMc|/bound   2 max |ΔPc|/boundP   3 max |ΔRc|/boundR
 *   4 max |ΔMm|/max(1, Mm)   5 max |ΔMm|/bound   6 max |ΔPm|/boundP   7 max |ΔRm|/boundR */
static inline double out_at(const void* a, int out_f64, int64_t i) {
    return out_f64 ? ((const double*)a)[i] : (double)((const float*)a)[i];
}

int oracle_sc_minn_check(const void* x, int is_c128, int64_t B, int64_t nb, int64_t T, int64_t N,
                         const void* Mc, const void* Pc, const void* Rc, const void* Mm, const void* Pm,
                         const void* Rm, int out_f64, double kP, double kR, double kM, double* stats,
                         int nthreads) {
    if (!x || B < 0 || nb < 1 || N < 4 || N % 4 || T < N || !Mc || !Pc || !Rc || !Mm || !Pm || !Rm || !stats)
        return -1;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    const int64_t nout = T - N + 1;
    const double u = 0x1p-24;
    int rc = 0;
#pragma omp parallel
    {
        ld* pre = (ld*)malloc(sizeof(ld) * 7 * (size_t)(T + 1));
        double* o = (double*)malloc(sizeof(double) * 8 * (size_t)nout);
        double* xd = (double*)malloc(sizeof(double) * 2 * (size_t)(nb * T));
        if (!pre || !o || !xd) {
#pragma omp atomic write
            rc = -2;
        }
#pragma omp for schedule(dynamic, 8)
        for (int64_t b = 0; b < B; ++b) {
            if (!pre || !o || !xd) continue;
            for (int64_t i = 0; i < 2 * nb * T; ++i)
                xd[i] = is_c128 ? ((const double*)x)[2 * b * nb * T + i] : (double)((const float*)x)[2 * b * nb * T + i];
            scm_ref_one(xd, nb, T, N, pre, o);
            double st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            for (int64_t d = 0; d < nout; ++d) {
                const int64_t g = b * nout + d;
                /* combined S&C */
                {
                    const double pr = o[d], pi = o[nout + d], R = o[2 * nout + d], S = o[3 * nout + d];
                    const double ap = hypot(pr, pi), Rm_ = R > 1e-12 ? R : 1e-12, M = ap * ap / (Rm_ * Rm_);
                    const double bP = kP * u * S + u * ap, bR = kR * u * R;
                    const double dP = hypot(out_at(Pc, out_f64, 2 * g) - pr, out_at(Pc, out_f64, 2 * g + 1) - pi);
                    const double dR = fabs(out_at(Rc, out_f64, g) - R), dM = fabs(out_at(Mc, out_f64, g) - M);
                    const double bM = fp32_metric_bound(ap, R, M, bP, bR, kM);
                    if (!(dM <= st[0])) st[0] = dM;                     /* NaN propagates as a failure */
                    if (!(dM / bM <= st[1])) st[1] = dM / bM;
                    if (!(dP / (bP + 1e-300) <= st[2])) st[2] = dP / (bP + 1e-300);
                    if (!(dR / (bR + 1e-300) <= st[3])) st[3] = dR / (bR + 1e-300);
                }
                /* Minn */
                {
                    const double pr = o[4 * nout + d], pi = o[5 * nout + d], R = o[6 * nout + d], S = o[7 * nout + d];
                    const double c = pr > 0.0 ? pr : 0.0, Rm_ = R > 1e-12 ? R : 1e-12, M = c * c / (Rm_ * Rm_);
                    const double bP = kP * u * S + u * hypot(pr, pi), bR = kR * u * R;
                    const double dP = hypot(out_at(Pm, out_f64, 2 * g) - pr, out_at(Pm, out_f64, 2 * g + 1) - pi);
                    const double dR = fabs(out_at(Rm, out_f64, g) - R), dM = fabs(out_at(Mm, out_f64, g) - M);
                    const double bM = fp32_metric_bound(c, R, M, bP, bR, kM);
                    const double rn = dM / (M > 1.0 ? M : 1.0);
                    if (!(rn <= st[4])) st[4] = rn;
                    if (!(dM / bM <= st[5])) st[5] = dM / bM;
                    if (!(dP / (bP + 1e-300) <= st[6])) st[6] = dP / (bP + 1e-300);
                    if (!(dR / (bR + 1e-300) <= st[7])) st[7] = dR / (bR + 1e-300);
                }
            }
            for (int k = 0; k < 8; ++k) stats[8 * b + k] = st[k];
        }
        free(pre); free(o); free(xd);
    }
    return rc;
}

/* In-place iterative radix-2 DIT FFT (fp64), N a power of two; tw[k] = exp(-2πi·k/N), k < N/2,
 * from libm cos/sin of exact index ratios.  Normwise relative error ~log2(N)·1e-16. */
static void fft_pow2(double* a, int64_t N, const double* tw) {
    for (int64_t i = 1, j = 0; i < N; ++i) {
        int64_t bit = N >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) {
            double t0 = a[2 * i], t1 = a[2 * i + 1];
            a[2 * i] = a[2 * j]; a[2 * i + 1] = a[2 * j + 1];
            a[2 * j] = t0; a[2 * j + 1] = t1;
        }
    }
    for (int64_t len = 2; len <= N; len <<= 1) {
        const int64_t h = len >> 1, step = N / len;
        for (int64_t s0 = 0; s0 < N; s0 += len) {
            for (int64_t k = 0; k < h; ++k) {
                const double wr = tw[2 * k * step], wi = tw[2 * k * step + 1];
                double* p = a + 2 * (s0 + k);
                double* q = a + 2 * (s0 + k + h);
                const double vr = q[0] * wr - q[1] * wi, vi = q[0] * wi + q[1] * wr;
                q[0] = p[0] - vr; q[1] = p[1] - vi;
                p[0] += vr; p[1] += vi;
            }
        }
    }
}

/* zc_freq.compute_frequency_metric (zc_freq.py:62-99) at every offset off in [0, T-(N+cp)]:
 *   window w = x[br][off+cp : off+cp+N];  b_j = fftshift(fft(w))[(N/2 + idx_j) % N] = DFT_N(w) at
 *   frequency idx_j mod N;  metric = |Σ_br Σ_j conj(t_j)·b_j|² / max(E_t·Σ_br Σ_j |b_j|², 1e-12).
 * The window's DFT in fp64: a radix-2 FFT for N a power of two (the reference's np.fft.fft), else a
 * direct DFT of the bins; twiddles from libm of exact index ratios.  Engine metric [B][noff] (fp32 if
 * is_f32 else fp64).  Error model of an fp32 FFT-based engine (eps = its normwise relative FFT error):
 *   ρ = ||Δb||/||b|| <= eps·sqrt(N)·||w||/||b||   (Parseval: ||ΔX|| <= eps·||X|| = eps·sqrt(N)·||w||)
 *   |Δm| <= 2·(sqrt(nb·m) + m)·ρ + (nb + 1)·ρ² + kM·u·m
 * (first-order perturbation of m = |<T, b>|² / (E_t·||b||²) over the nb·62 gathered bins, plus the
 * metric's own fp32 operations).  stats [B][3]: 0 max|Δm|, 1 max |Δm|/bound, 2 max oracle metric. */
int oracle_zc_freq_check(const void* x, int is_c128, int64_t B, int64_t nb, int64_t T, int64_t N, int64_t cp,
                         int32_t nbins, const int32_t* idx, const double* tmpl, double tmpl_energy,
                         const void* eng, int is_f32, double eps, double kM, double* stats, int nthreads) {
    if (!x || B < 0 || nb < 1 || N < 2 || cp < 0 || T < N + cp || nbins < 1 || !idx || !tmpl || !eng || !stats)
        return -1;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    const int64_t noff = T - (N + cp) + 1;
    const int pow2 = (N & (N - 1)) == 0;
    double* tw = (double*)malloc(sizeof(double) * (pow2 ? (size_t)N : 2 * (size_t)nbins * (size_t)N));
    if (!tw) return -2;
    if (pow2) {
        for (int64_t k = 0; k < N / 2; ++k) {
            const double a = -2.0 * M_PI * (double)k / (double)N;
            tw[2 * k] = cos(a);
            tw[2 * k + 1] = sin(a);
        }
    } else {
        for (int j = 0; j < nbins; ++j) {
            const int64_t k = ((int64_t)idx[j] % N + N) % N;
            for (int64_t n = 0; n < N; ++n) {
                const double a = -2.0 * M_PI * (double)((k * n) % N) / (double)N;
                tw[2 * ((int64_t)j * N + n)] = cos(a);
                tw[2 * ((int64_t)j * N + n) + 1] = sin(a);
            }
        }
    }
    int rc = 0;
#pragma omp parallel
    {
        double* w = (double*)malloc(sizeof(double) * 2 * (size_t)N);
        if (!w) {
#pragma omp atomic write
            rc = -2;
        }
#pragma omp for schedule(dynamic, 64)
        for (int64_t b = 0; b < B; ++b) {
            if (!w) continue;
            double st[3] = {0, 0, 0};
            for (int64_t off = 0; off < noff; ++off) {
                double sr = 0, si = 0, D = 0, W2 = 0;
                for (int64_t br = 0; br < nb; ++br) {
                    const int64_t base = (b * nb + br) * T + off + cp;
                    for (int64_t n = 0; n < N; ++n) {
                        w[2 * n] = is_c128 ? ((const double*)x)[2 * (base + n)] : (double)((const float*)x)[2 * (base + n)];
                        w[2 * n + 1] = is_c128 ? ((const double*)x)[2 * (base + n) + 1]
                                               : (double)((const float*)x)[2 * (base + n) + 1];
                        W2 += w[2 * n] * w[2 * n] + w[2 * n + 1] * w[2 * n + 1];
                    }
                    if (pow2) fft_pow2(w, N, tw);
                    for (int j = 0; j < nbins; ++j) {
                        double br_ = 0, bi_ = 0;
                        if (pow2) {
                            const int64_t k = ((int64_t)idx[j] % N + N) % N;
                            br_ = w[2 * k]; bi_ = w[2 * k + 1];
                        } else {
                            const double* t = tw + 2 * (int64_t)j * N;
                            for (int64_t n = 0; n < N; ++n) {
                                br_ += w[2 * n] * t[2 * n] - w[2 * n + 1] * t[2 * n + 1];
                                bi_ += w[2 * n] * t[2 * n + 1] + w[2 * n + 1] * t[2 * n];
                            }
                        }
                        /* conj(t_j)·b_j  (np.vdot conjugates its first argument, zc_freq.py:95) */
                        sr += tmpl[2 * j] * br_ + tmpl[2 * j + 1] * bi_;
                        si += tmpl[2 * j] * bi_ - tmpl[2 * j + 1] * br_;
                        D += br_ * br_ + bi_ * bi_;
                    }
                }
                const double den = tmpl_energy * D;
                const double m = (sr * sr + si * si) / (den > 1e-12 ? den : 1e-12);
                const double e = is_f32 ? (double)((const float*)eng)[b * noff + off] : ((const double*)eng)[b * noff + off];
                const double dm = fabs(e - m);
                const double rho = D > 0 ? eps * sqrt((double)N) * sqrt(W2) / sqrt(D) : INFINITY;
                const double bound = 2.0 * (sqrt((double)nb * m) + m) * rho + (double)(nb + 1) * rho * rho +
                                     kM * 0x1p-24 * m + 1e-300;
                if (!(dm <= st[0])) st[0] = dm;
                if (!(dm / bound <= st[1])) st[1] = dm / bound;
                if (m > st[2]) st[2] = m;
            }
            for (int k = 0; k < 3; ++k) stats[3 * b + k] = st[k];
        }
        free(w);
    }
    free(tw);
    return rc;
}
