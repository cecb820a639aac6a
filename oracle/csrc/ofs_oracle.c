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
