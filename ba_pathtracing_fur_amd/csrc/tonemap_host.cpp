// tonemap_host.cpp -- the host part of the tonemapped output stage: KIRK's
// sequential float running sum of the per-pixel log luminances.
//
// Tonemapper::RGB_to_Yxy (Tonemapping.cpp:66-91) keeps `float sum` and adds
// `log(2.3e-5 + Y)` -- a double -- pixel by pixel:  s <- (float)((double)s + l).
// Every step rounds to float, so the result depends on the order and no
// reassociation reproduces it; the chain has to be walked in pixel order.  One
// step as written is three dependent operations (convert, add, convert); here
// it is ONE double add on a shifted value, checked afterwards:
//
//   While s stays in one float binade [2^(e-1), 2^e), float rounding is rounding
//   to the grid 2^(e-24).  With C = sign(s) 2^(e+28), u = C + s is exact and lies
//   in a double binade whose ulp is that same grid, so u + l rounds C + s + l to
//   the float grid in one double add (ties to even agree: C/ulp = 2^52 is even).
//   This equals KIRK's step except where the double rounding of (double)s + l
//   lands on a float midpoint, or where s leaves the binade.
//
// So a block of steps is run with the one-add chain, then every step of it is
// re-checked against KIRK's expression (independent operations: vectorised),
// and from the first step that differs the block restarts with KIRK's step.
// The result is KIRK's sum bit for bit by induction; the check costs no
// dependent latency.  tests/test_output.py compares it with the plain loop.
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstring>

#include "scene.h"

namespace khp {

static inline float kirk_step(float s, double l) { return (float)((double)s + l); }

float log_sum_feed(float s, const double* l, size_t n) {
    constexpr size_t B = 2048;
    double buf[B + 1];
    size_t k = 0;
    while (k < n) {
        const size_t m = n - k < B ? n - k : B;
        if (s != s) return s;  // NaN absorbs every later term (x86 keeps the first operand's NaN)
        if (std::isinf(s)) {
            // +-inf stays itself until a NaN or the opposite infinity turns it into NaN
            // (an inf pixel blacks out KIRK's whole texture; its frame must not cost a
            // step per remaining pixel)
            for (; k < n; ++k)
                if (l[k] != l[k] || l[k] == (double)-s) return kirk_step(s, l[k]);
            return s;
        }
        if (s == 0.0f) {  // no binade yet: KIRK's step as written
            s = kirk_step(s, l[k]);
            ++k;
            continue;
        }
        int e;
        (void)std::frexp(s, &e);   // |s| in [2^(e-1), 2^e)
        const double C = std::copysign(std::ldexp(1.0, e + 28), (double)s);
        const double* lk = l + k;
        double u = C + (double)s;  // exact
        buf[0] = (double)s;
        for (size_t j = 0; j < m; ++j) {  // the chain: one double add per step
            u = u + lk[j];
            buf[j + 1] = u;
        }
        for (size_t j = 1; j <= m; ++j) buf[j] -= C;  // exact: same sign and binade as C
        int bad = 0;
        for (size_t j = 0; j < m; ++j) bad |= (double)kirk_step((float)buf[j], lk[j]) != buf[j + 1];
        if (!bad) {
            s = (float)buf[m];
            k += m;
            continue;
        }
        size_t j = 0;  // buf[j] is KIRK's value; step j is the first that differs
        while ((double)kirk_step((float)buf[j], lk[j]) == buf[j + 1]) ++j;
        s = kirk_step((float)buf[j], lk[j]);
        k += j + 1;
    }
    return s;
}

}  // namespace khp

extern "C" khp_status khp_tonemap_log_sum(const double* terms, uint64_t n, float start, float* out) {
    if ((!terms && n) || !out) return khp::fail(KHP_EINVAL, "khp_tonemap_log_sum: null argument");
    *out = khp::log_sum_feed(start, terms, (size_t)n);
    return KHP_OK;
}
