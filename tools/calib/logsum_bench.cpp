// Calibration (dev tool): KIRK's sequential float log-luminance sum over a 1080p
// frame's 2,073,600 double terms -- the plain loop, the one-add chain with
// verification (tonemap_host.cpp) and an integer-grid prefix-sum form -- timed
// on this host's CPU.  Build: g++ -O3 -march=x86-64-v3 -ffp-contract=off.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>
#include <random>
#include <chrono>
#include <algorithm>
static inline float step_exact(float s, double l) { return (float)((double)s + l); }
float slow_sum(const double* l, size_t n) { float s = 0.0f; for (size_t k = 0; k < n; ++k) s = step_exact(s, l[k]); return s; }
size_t nslow = 0;
// integer-grid formulation: within a binade, KIRK's step (bar double-rounding ties) is
// U <- U + rint(l/g) on the grid g = ulp(s); exact integer adds associate, so the prefix
// sums are computed in independent 64-element chains; every step is then verified.
float fast_sum2(const double* l, size_t n, float s) {
    constexpr size_t B = 4096, C = 64;
    alignas(64) double buf[B + 1];
    size_t k = 0;
    while (k < n) {
        const size_t m = std::min(B, n - k);
        if (s == 0.0f || !std::isfinite(s)) { s = step_exact(s, l[k]); ++k; ++nslow; continue; }
        int e;
        std::frexp(s, &e);
        const double g = std::ldexp(1.0, e - 24), ig = std::ldexp(1.0, 24 - e);
        const double* lk = l + k;
        for (size_t j = 0; j < m; ++j) buf[j + 1] = std::nearbyint(lk[j] * ig);   // R_j (exact scaling)
        // exact integer sums associate: chunk totals (independent), their prefix, then
        // each chunk's running sums from its own carry (independent chains)
        double carry[B / C + 1];
        carry[0] = (double)s * ig;   // U_0, exact integer
        buf[0] = carry[0];
        const size_t nc = (m + C - 1) / C;
        for (size_t c = 0; c < nc; ++c) {
            const size_t c0 = c * C, c1 = std::min(m, c0 + C);
            double t0 = 0, t1 = 0, t2 = 0, t3 = 0;
            size_t j = c0;
            for (; j + 4 <= c1; j += 4) { t0 += buf[j + 1]; t1 += buf[j + 2]; t2 += buf[j + 3]; t3 += buf[j + 4]; }
            for (; j < c1; ++j) t0 += buf[j + 1];
            carry[c + 1] = carry[c] + ((t0 + t1) + (t2 + t3));
        }
        for (size_t c = 0; c < nc; ++c) {
            const size_t c0 = c * C, c1 = std::min(m, c0 + C);
            double acc = carry[c];
            for (size_t j = c0; j < c1; ++j) { acc += buf[j + 1]; buf[j + 1] = acc; }
        }
        for (size_t j = 0; j <= m; ++j) buf[j] *= g;   // back to s values (exact)
        int bad = 0;
        for (size_t j = 0; j < m; ++j) bad |= (double)(float)(buf[j] + lk[j]) != buf[j + 1];
        if (!bad) { s = (float)buf[m]; k += m; continue; }
        size_t j = 0;
        while ((double)(float)(buf[j] + lk[j]) == buf[j + 1]) ++j;
        s = step_exact((float)buf[j], lk[j]);
        k += j + 1;
        ++nslow;
    }
    return s;
}
float fast_sum(const double* l, size_t n, float s) {
    constexpr size_t B = 2048;
    double buf[B + 1];
    size_t k = 0;
    while (k < n) {
        const size_t m = std::min(B, n - k);
        const float s0 = s;
        if (s0 == 0.0f || !std::isfinite(s0)) { s = step_exact(s0, l[k]); ++k; ++nslow; continue; }
        int e;
        std::frexp(s0, &e);
        const double C = std::copysign(std::ldexp(1.0, e + 28), (double)s0);
        double u = C + (double)s0;
        buf[0] = (double)s0;
        const double* lk = l + k;
        for (size_t j = 0; j < m; ++j) { u = u + lk[j]; buf[j + 1] = u - C; }
        int bad = 0;
        for (size_t j = 0; j < m; ++j) bad |= (double)(float)(buf[j] + lk[j]) != buf[j + 1];
        if (!bad) { s = (float)buf[m]; k += m; continue; }
        size_t j = 0;
        while ((double)(float)(buf[j] + lk[j]) == buf[j + 1]) ++j;
        s = step_exact((float)buf[j], lk[j]);
        k += j + 1;
        ++nslow;
    }
    return s;
}
int main() {
    const size_t n = 1920 * 1080;
    std::vector<double> l(n);
    std::mt19937 rng(1);
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    for (int trial = 0; trial < 4; ++trial) {
        for (size_t i = 0; i < n; ++i) {
            float Y = trial == 0 ? U(rng) : trial == 1 ? U(rng) * U(rng) * 3.0f : trial == 2 ? (U(rng) < 0.3f ? 0.0f : U(rng) * 0.1f) : std::exp(8.0f * (U(rng) - 0.5f));
            l[i] = std::log(2.3e-5 + (double)Y);
        }
        for (int rep = 0; rep < 3; ++rep) {
        auto t0 = std::chrono::steady_clock::now();
        float a = slow_sum(l.data(), n);
        auto t1 = std::chrono::steady_clock::now();
        float c = fast_sum(l.data(), n, 0.0f);
        auto t2 = std::chrono::steady_clock::now();
        nslow = 0;
        float b = fast_sum2(l.data(), n, 0.0f);
        auto t3 = std::chrono::steady_clock::now();
        printf("trial %d slow %.3f ms chain %.3f ms grid %.3f ms  %s %s nslow=%zu\n", trial, std::chrono::duration<double, std::milli>(t1 - t0).count(),
               std::chrono::duration<double, std::milli>(t2 - t1).count(), std::chrono::duration<double, std::milli>(t3 - t2).count(),
               memcmp(&a, &c, 4) == 0 ? "EQUAL" : "DIFF", memcmp(&a, &b, 4) == 0 ? "EQUAL" : "DIFF", nslow);
        }
    }
}
