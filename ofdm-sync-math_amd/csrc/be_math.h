// Lean fp64 sin/cos and atan2 for the fast receiver back-end (backend.hip).
//
// The ocml versions carry large-argument and special-case paths whose registers the compiler keeps
// across the kernel's whole frame loop (40 VGPRs for atan2, 26 for sincos at the fast kernel's
// peak, r05aa): with them the kernel needs 243 VGPRs, two workgroups per CU; without them it fits
// the 168 of three.  These follow the published fdlibm algorithms (s_sin.c/k_sin.c/k_cos.c,
// e_atan2.c/s_atan.c: same minimax coefficients), reshaped branch-free:
//  * sincos: three-term Cody-Waite reduction by pi/2 with FMAs (exact-rounded for |x| up to ~2^40;
//    the window tones reach |x| < pi·2^31), then the k_sin / k_cos polynomials on |r| <= pi/4;
//  * atan2: one division - z = num/den with the (7/16, 11/16) argument reduction folded into the
//    numerator and denominator - the s_atan polynomial, then octant / quadrant corrections with
//    two-part pi/2 and pi.
// Against glibc over the tested ranges: atan2 within 1 ulp, sin/cos within 1.1e-16 absolute (1 ulp,
// 2 next to a zero) - tests/test_be_math.py compiles this header for the host and compares.
#pragma once

#ifndef __HIPCC__
#include <cmath>
#define OFS_HD
#else
#define OFS_HD __host__ __device__
#endif

namespace ofs_bemath {
#ifndef __HIPCC__
using std::fabs; using std::floor; using std::fma; using std::rint; using std::signbit;
#endif

// an fp64 constant materialised into scalar registers by the instructions at its use: without this
// the compiler hoists every coefficient out of the kernel's frame loop into a VGPR pair held across
// it (r05ab: ~50 VGPRs of polynomial coefficients), and with the materialisation outside the asm it
// hoists the scalar moves instead and spills the SGPRs to VGPR lanes (a v_readlane per use)
#if defined(__HIP_DEVICE_COMPILE__)
template <unsigned long long B>
__device__ __forceinline__ double kd_() {
    unsigned lo, hi;
    asm volatile("s_mov_b32 %0, %2\n\ts_mov_b32 %1, %3"
                 : "=s"(lo), "=s"(hi) : "i"((unsigned)(B & 0xffffffffu)), "i"((unsigned)(B >> 32)));
    return __hiloint2double((int)hi, (int)lo);
}
#define OFS_BEMATH_K(c) ofs_bemath::kd_<__builtin_bit_cast(unsigned long long, (double)(c))>()
// a·b + c with the constant c read from its scalar pair by the VOP3 form: the compiler otherwise
// picks v_fmac_f64, whose addend is the destination, and copies every constant into VGPRs first
// (two v_mov_b32 per Horner step)
__device__ __forceinline__ double fmak(double a, double b, double c) {
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
}
#else
#define OFS_BEMATH_K(c) (c)
inline double fmak(double a, double b, double c) { return fma(a, b, c); }
#endif

OFS_HD inline void sincos_lean(double x, double* s, double* c) {
    const double n = rint(x * OFS_BEMATH_K(0.63661977236758134308));             // 2/pi
    double r = fma(-n, OFS_BEMATH_K(1.5707963267948966), x);                     // pi/2 = P1 + P2 + P3
    r = fma(-n, OFS_BEMATH_K(6.123233995736766e-17), r);
    r = fma(-n, OFS_BEMATH_K(-1.4973849048591698e-33), r);
    const double z = r * r;
    double ps = fma(z, OFS_BEMATH_K(1.58969099521155010221e-10), OFS_BEMATH_K(-2.50507602534068634195e-08));
    ps = fmak(z, ps, OFS_BEMATH_K(2.75573137070700676789e-06));
    ps = fmak(z, ps, OFS_BEMATH_K(-1.98412698298579493134e-04));
    ps = fmak(z, ps, OFS_BEMATH_K(8.33333333332248946124e-03));
    const double sn = r + (z * r) * fmak(z, ps, OFS_BEMATH_K(-1.66666666666666324348e-01));
    double pc = fma(z, OFS_BEMATH_K(-1.13596475577881948265e-11), OFS_BEMATH_K(2.08757232129817482790e-09));
    pc = fmak(z, pc, OFS_BEMATH_K(-2.75573143513906633035e-07));
    pc = fmak(z, pc, OFS_BEMATH_K(2.48015872894767294178e-05));
    pc = fmak(z, pc, OFS_BEMATH_K(-1.38888888888741095749e-03));
    pc = z * fmak(z, pc, OFS_BEMATH_K(4.16666666666666019037e-02));
    const double hz = 0.5 * z, w = 1.0 - hz;
    const double cn = w + (((1.0 - w) - hz) + z * pc);
    const double q = n - 4.0 * floor(n * 0.25);                       // quadrant 0..3 (exact)
    const bool odd = q == 1.0 || q == 3.0;
    const double s0 = odd ? cn : sn, c0 = odd ? sn : cn;
    *s = (q >= 2.0) ? -s0 : s0;                                       // q: (s, c) (c, -s) (-s, -c) (-c, s)
    *c = (q == 1.0 || q == 2.0) ? -c0 : c0;
}

OFS_HD inline double atan2_lean(double y, double x) {
    const double ax = fabs(x), ay = fabs(y);
    const bool sw = ay > ax;                                          // |y/x| > 1: pi/2 - atan(|x/y|)
    const double num = sw ? ax : ay, den = sw ? ay : ax;
    const bool r0 = num * 16.0 < 7.0 * den || den == 0.0;             // t = num/den < 7/16 (or 0/0)
    const bool r1 = !r0 && num * 16.0 < 11.0 * den;                   // 7/16 <= t < 11/16: atan(1/2) + ...
    const double nn = r0 ? num : (r1 ? 2.0 * num - den : num - den);  // else: atan(1) + atan((t-1)/(t+1))
    const double dd = den == 0.0 ? 1.0 : (r0 ? den : (r1 ? 2.0 * den + num : num + den));
    const double z = nn / dd, z2 = z * z, w = z2 * z2;
    double s1 = fma(w, OFS_BEMATH_K(1.62858201153657823623e-02), OFS_BEMATH_K(4.97687799461593236017e-02));
    s1 = fmak(w, s1, OFS_BEMATH_K(6.66107313738753120669e-02));
    s1 = fmak(w, s1, OFS_BEMATH_K(9.09088713343650656196e-02));
    s1 = fmak(w, s1, OFS_BEMATH_K(1.42857142725034663711e-01));
    s1 = z2 * fmak(w, s1, OFS_BEMATH_K(3.33333333333329318027e-01));
    double s2 = fma(w, OFS_BEMATH_K(-3.65315727442169155270e-02), OFS_BEMATH_K(-5.83357013379057348645e-02));
    s2 = fmak(w, s2, OFS_BEMATH_K(-7.69187620504482999495e-02));
    s2 = fmak(w, s2, OFS_BEMATH_K(-1.11111104054623557880e-01));
    s2 = w * fmak(w, s2, OFS_BEMATH_K(-1.99999999998764832476e-01));
    const double zs = z * (s1 + s2);
    const double hi = r1 ? OFS_BEMATH_K(4.63647609000806093515e-01) : OFS_BEMATH_K(7.85398163397448278999e-01);
    const double lo = r1 ? OFS_BEMATH_K(2.26987774529616870924e-17) : OFS_BEMATH_K(3.06161699786838301793e-17);
    double a = r0 ? z - zs : hi - ((zs - lo) - z);                    // atan(num/den) in [0, pi/4]
    const bool xn = signbit(x);
    if (sw || xn) {                       // pi/2 - a, pi - a, or (|y| > |x|, x < 0) pi/2 + a; two-part constants
        const double bh = sw ? OFS_BEMATH_K(1.5707963267948966) : OFS_BEMATH_K(3.141592653589793);
        const double bl = sw ? OFS_BEMATH_K(6.123233995736766e-17) : OFS_BEMATH_K(1.2246467991473532e-16);
        a = (sw && xn) ? bh + (a + bl) : bh - (a - bl);
    }
    return signbit(y) ? -a : a;
}

}  // namespace ofs_bemath
