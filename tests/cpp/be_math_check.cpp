// Host check of the back-end's lean fp64 sin/cos and atan2 (csrc/be_math.h) against glibc:
// prints the largest error in ulps per function and range.  Built and run by tests/test_be_math.py.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>

#include "be_math.h"

static double ulps(double got, double ref) {
    if (std::isnan(ref)) return std::isnan(got) ? 0.0 : 1e300;
    if (got == ref) return 0.0;
    const double sp = std::nextafter(std::fabs(ref), INFINITY) - std::fabs(ref);
    return std::fabs(got - ref) / sp;
}

int main() {
    std::mt19937_64 g(2026);
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    std::normal_distribution<double> nd(0.0, 1.0);
    const double scales[] = {1e-6, 1.0, 100.0, 1e4, 1e6, 6.7e9};
    for (double sc : scales) {
        double es = 0, ec = 0, abs_s = 0, abs_c = 0;
        for (int i = 0; i < 400000; ++i) {
            const double x = u(g) * sc;
            double s, c;
            ofs_bemath::sincos_lean(x, &s, &c);
            es = std::fmax(es, ulps(s, std::sin(x)));
            ec = std::fmax(ec, ulps(c, std::cos(x)));
            abs_s = std::fmax(abs_s, std::fabs(s - std::sin(x)));
            abs_c = std::fmax(abs_c, std::fabs(c - std::cos(x)));
        }
        std::printf("sincos %g %.3f %.3f %.3g %.3g\n", sc, es, ec, abs_s, abs_c);
    }
    const double ysc[] = {1e-9, 1e-3, 1.0, 1e3, 1e9};
    for (double sc : ysc) {
        double e = 0;
        for (int i = 0; i < 400000; ++i) {
            const double y = nd(g) * sc, x = nd(g);
            e = std::fmax(e, ulps(ofs_bemath::atan2_lean(y, x), std::atan2(y, x)));
        }
        std::printf("atan2 %g %.3f\n", sc, e);
    }
    // signed zeros, axes, diagonals
    const double sp[][2] = {{0.0, 1.0}, {0.0, -1.0}, {-0.0, 1.0}, {-0.0, -1.0}, {1.0, 0.0}, {-1.0, 0.0},
                            {1.0, -0.0}, {0.0, 0.0}, {-0.0, -0.0}, {0.0, -0.0}, {1.0, 1.0}, {-1.0, -1.0},
                            {1.0, -1.0}, {3.0, 4.0}, {1e-300, 1.0}, {1.0, 1e-300}};
    double e = 0;
    for (auto& p : sp) e = std::fmax(e, ulps(ofs_bemath::atan2_lean(p[0], p[1]), std::atan2(p[0], p[1])));
    std::printf("atan2_special 0 %.3f\n", e);
    return 0;
}
