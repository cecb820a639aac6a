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

int oracle_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
