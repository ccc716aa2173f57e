// wost_tables.cpp -- see wost_tables.h.
#include "wost_tables.h"

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>
#include <cmath>

namespace wost {

namespace {

// f(i) for i in [0, n) on up to 8 host threads taking chunks of kChunk indices (the sampler
// tables' nodes and density samples are independent of one another: the same bits as one
// thread; a fresh process's first delta-tracking solve waited ~60 ms for them on one core).
template <class F>
void parallel_for(int n, F f, int kChunk = 64) {
#if defined(WOST_TABLES_SERIAL)   // (tests/test_tables_parallel.py: the one-thread reference)
    const int T = 1;
#else
    const unsigned hw = std::thread::hardware_concurrency();
    const int T = (int)std::max(1u, std::min(8u, hw));
#endif
    if (T <= 1 || n < 4 * kChunk) {
        for (int i = 0; i < n; ++i) f(i);
        return;
    }
    std::atomic<int> next{0};
    auto work = [&]() {
        for (;;) {
            const int i0 = next.fetch_add(kChunk);
            if (i0 >= n) return;
            for (int i = i0; i < std::min(n, i0 + kChunk); ++i) f(i);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(work);
    work();
    for (std::thread& x : th) x.join();
}

}  // namespace

static const double kPi = 3.14159265358979323846;

double i0e_host(double x) {
    x = std::fabs(x);
    if (x == 0.0) return 1.0;
    // integrand peaks at t = 0 with width ~ 1/sqrt(x); 4096 panels resolve
    // x up to ~1e5, beyond that use the asymptotic series.
    if (x > 1.0e5) {
        double s = 1.0, term = 1.0;
        for (int k = 1; k < 12; ++k) {
            term *= (2.0 * k - 1.0) * (2.0 * k - 1.0) / (8.0 * k * x);
            s += term;
        }
        return s / std::sqrt(2.0 * kPi * x);
    }
    const int m = 4096;
    const double h = kPi / m;
    double acc = 0.5 * (1.0 + std::exp(-2.0 * x));
    for (int j = 1; j < m; ++j) acc += std::exp(x * (std::cos(j * h) - 1.0));
    return acc * h / kPi;
}

double i0_host(double x) { return i0e_host(x) * std::exp(std::fabs(x)); }

double k0_host(double x) {
    if (x <= 0.0) return INFINITY;
    if (x <= 2.0) {
        // K0(x) = -(ln(x/2) + gamma) I0(x) + sum_{k>=1} (x^2/4)^k / (k!)^2 H_k
        const double gamma = 0.57721566490153286061;
        const double q = 0.25 * x * x;
        double term = 1.0, i0 = 1.0, s = 0.0, hk = 0.0;
        for (int k = 1; k < 40; ++k) {
            term *= q / ((double)k * k);
            hk += 1.0 / k;
            i0 += term;
            s += term * hk;
        }
        return -(std::log(0.5 * x) + gamma) * i0 + s;
    }
    // K0(x) = int_0^inf exp(-x cosh t) dt, trapezoid (spectrally accurate).
    const double h = 0.02;
    double acc = 0.5 * std::exp(-x);
    for (int j = 1;; ++j) {
        double v = std::exp(-x * std::cosh(j * h));
        acc += v;
        if (v < 1e-300 || (v < 1e-18 * acc)) break;
    }
    return acc * h;
}

static void cheb_fit(double (*g)(double), float* c, int n) {
    std::vector<double> f(n);
    for (int j = 0; j < n; ++j) f[j] = g(std::cos(kPi * (j + 0.5) / n));
    for (int k = 0; k < n; ++k) {
        double s = 0.0;
        for (int j = 0; j < n; ++j) s += f[j] * std::cos(kPi * k * (j + 0.5) / n);
        s *= 2.0 / n;
        if (k == 0) s *= 0.5;
        c[k] = (float)s;
    }
}

static double g_region_a(double t) { return i0e_host(4.0 * (t + 1.0)); }
static double g_region_b(double t) {
    double x = 16.0 / (t + 1.0);
    return std::sqrt(x) * i0e_host(x);
}

void fit_i0e_chebyshev(float* ca, int na, float* cb, int nb) {
    cheb_fit(g_region_a, ca, na);
    cheb_fit(g_region_b, cb, nb);
}

double screened_greens_norm(double R, double sigma_bar) {
    double x = R * std::sqrt(sigma_bar);
    // 1/I0(x) = exp(-x)/i0e(x)
    return (1.0 / sigma_bar) * (1.0 - std::exp(-x) / i0e_host(x));
}

double screened_greens(double r, double R, double sigma_bar) {
    const double s = std::sqrt(sigma_bar);
    const double kR = k0_host(R * s), iR = i0_host(R * s);
    return (k0_host(r * s) - (kR / iR) * i0_host(r * s)) / (2.0 * kPi);
}

void greens_phi(double x, double* phi, double* dphi) {
    // q = x^2/4; I0 = sum q^k/(k!)^2; A = (I0 - 1)/q = sum_{k>=1} q^(k-1)/(k!)^2;
    // Phi = A / (4 I0). dA/dx = (x/2) sum_{k>=2} (k-1) q^(k-2)/(k!)^2; I1 = (x/2) sum q^k/(k!(k+1)!)
    const double q = 0.25 * x * x;
    double i0 = 1.0, A = 0.0, dAq = 0.0, s1 = 0.0;
    double t = 1.0;        // q^k / (k!)^2
    double tq = 1.0;       // q^(k-1) / (k!)^2 (k >= 1)
    double tqq = 0.0;      // q^(k-2) / (k!)^2 (k >= 2)
    s1 = 1.0;              // k = 0 term of sum q^k/(k!(k+1)!)
    for (int k = 1; k < 200; ++k) {
        const double kk = (double)k * k;
        t = t * q / kk;
        tq = (k == 1) ? 1.0 : tq * q / kk;
        tqq = (k == 2) ? 0.25 : (k > 2 ? tqq * q / kk : 0.0);
        i0 += t;
        A += tq;
        dAq += (k - 1) * tqq;
        s1 += t / (k + 1);
        if (t < 1e-18 * i0 && k > 4) break;
    }
    const double i1 = 0.5 * x * s1;
    const double dA = 0.5 * x * dAq;
    *phi = A / (4.0 * i0);
    *dphi = (dA * i0 - A * i1) / (4.0 * i0 * i0);
}

void greens_norm_cells(float* out, int cells, double xmax) {
    const double h = xmax / cells;
    for (int c = 0; c < cells; ++c) {
        double p0, d0, p1, d1;
        greens_phi(c * h, &p0, &d0);
        greens_phi((c + 1) * h, &p1, &d1);
        const double m0 = h * d0, m1 = h * d1;
        out[4 * c + 0] = (float)p0;
        out[4 * c + 1] = (float)m0;
        out[4 * c + 2] = (float)(3.0 * (p1 - p0) - 2.0 * m0 - m1);
        out[4 * c + 3] = (float)(2.0 * (p0 - p1) + m0 + m1);
    }
}

void greens_sampler_nodes(float* out, int n) {
    const double a = 1e-6;
    const double c0 = a - a * std::log(a);
    const double z = 1.0 - c0;
    auto cdf = [&](double rho) { return (rho - rho * std::log(rho) - c0) / z; };
    parallel_for(n, [&](int i) {
        const double u = (double)i / (double)(n - 1);
        double lo = a, hi = 1.0;
        if (i == 0) { out[i] = (float)a; return; }
        if (i == n - 1) { out[i] = 1.0f; return; }
        for (int it = 0; it < 200 && hi - lo > 1e-17; ++it) {
            double mid = 0.5 * (lo + hi);
            if (mid == lo || mid == hi) break;   // adjacent doubles: the bracket no longer moves
            if (cdf(mid) < u) lo = mid; else hi = mid;
        }
        out[i] = (float)(0.5 * (lo + hi));
    });
}

void greens_sampler_nodes_jacobian(float* out, int n) {
    auto cdf = [](double rho) { return rho * rho * (1.0 - 2.0 * std::log(rho)); };
    parallel_for(n, [&](int i) {
        const double u = (double)i / (double)(n - 1);
        if (i == 0) { out[i] = 0.0f; return; }
        if (i == n - 1) { out[i] = 1.0f; return; }
        double lo = 0.0, hi = 1.0;
        for (int it = 0; it < 200 && hi - lo > 1e-17; ++it) {
            const double mid = 0.5 * (lo + hi);
            if (mid == lo || mid == hi) break;   // adjacent doubles: the bracket no longer moves
            if (cdf(mid) < u) lo = mid; else hi = mid;
        }
        out[i] = (float)(0.5 * (lo + hi));
    });
}

// I0 by its power series (every term positive: no cancellation, ~1 ulp) for x <= 30, where it
// needs at most ~60 terms; i0_host's 4,096-panel quadrature otherwise. The sampler's
// 65,537 density samples took 2.4 s of host time per handle through the quadrature -- the
// whole cold start of a delta-tracking solve (bench.py "cold", profiles/r06_s1/).
static double i0_series(double x) {
    x = std::fabs(x);
    if (x > 30.0) return i0_host(x);
    const double q = 0.25 * x * x;
    double term = 1.0, s = 1.0;
    for (int k = 1; k < 200; ++k) {
        term *= q / ((double)k * (double)k);
        s += term;
        if (term < 1e-17 * s) break;
    }
    return s;
}

void screened_sampler_nodes(float* out, int n, double sigma_bar) {
    const double a = 1e-6;
    const int J = 1 << 16;
    const double h = (1.0 - a) / J;
    const double M = screened_greens_norm(1.0, sigma_bar);
    const double s = std::sqrt(sigma_bar);
    const double kR = k0_host(s), iR = i0_host(s);
    const double ratio = kR / iR;
    std::vector<double> p(J + 1), C(J + 1);
    parallel_for(J + 1, [&](int j) {
        const double rho = a + j * h;
        const double g = std::fabs((k0_host(rho * s) - ratio * i0_series(rho * s)) / (2.0 * kPi));
        p[j] = std::min(g, M);
    });
    C[0] = 0.0;
    for (int j = 0; j < J; ++j) C[j + 1] = C[j] + 0.5 * h * (p[j] + p[j + 1]);
    const double tot = C[J];
    parallel_for(n, [&](int i) {
        if (i == 0) { out[i] = (float)a; return; }
        if (i == n - 1) { out[i] = 1.0f; return; }
        const double target = tot * (double)i / (double)(n - 1);
        int j = (int)(std::upper_bound(C.begin(), C.end(), target) - C.begin()) - 1;
        j = std::max(0, std::min(j, J - 1));
        // density linear in the cell -> CDF quadratic: A d^2 + B d = T
        const double A = (p[j + 1] - p[j]) / (2.0 * h), B = p[j], T = target - C[j];
        const double disc = std::sqrt(std::max(0.0, B * B + 4.0 * A * T));
        const double d = (B + disc) > 0.0 ? 2.0 * T / (B + disc) : 0.0;
        out[i] = (float)(a + j * h + d);
    });
}

// ---------------------------------------------------------------------------
// compat="fixed" screened sampler (quirks Q4/Q5 corrected). A point y sampled
// from the ball's screened Green's function G(x, y; R) (2-D, sigma_bar) has
// radius rho R with, for the shape parameter s = R sqrt(sigma_bar),
//   p_s(rho) ~ rho [K0(rho s) - c I0(rho s)],  c = K0(s) / I0(s),
// whose CDF is closed-form (d/dt[-t K1(t)] = t K0(t), d/dt[t I1(t)] = t I0(t),
// and the Wronskian I0 K1 + I1 K0 = 1/s for the normaliser):
//   F_s(rho) = (1 - t K1(t) - c t I1(t)) / (1 - 1/I0(s)),  t = rho s.
// s -> 0 gives the Laplace law rho^2 (1 + 2 ln(1/rho)).
// ---------------------------------------------------------------------------
static void bessel_i01(double t, double* i0, double* i1) {
    // power series; every term is positive (no cancellation) and t <= kFixSMax
    const double q = 0.25 * t * t;
    double a = 1.0, b = 0.5 * t, s0 = a, s1 = b;
    for (int k = 1; k < 400; ++k) {
        a *= q / ((double)k * k);
        b *= q / ((double)k * (k + 1));
        s0 += a;
        s1 += b;
        if (a <= 1e-18 * s0 && b <= 1e-18 * s1) break;
    }
    *i0 = s0;
    *i1 = s1;
}

static void bessel_k01(double t, double* k0, double* k1) {
    if (t <= 2.0) {
        // A&S 9.6.13 / 9.6.11: K0 = -(ln(t/2) + gamma) I0 + sum q^k/(k!)^2 H_k,
        // K1 = 1/t + ln(t/2) I1 - (t/4) sum (psi(k+1) + psi(k+2)) q^k / (k! (k+1)!)
        const double gamma = 0.57721566490153286061;
        double i0, i1;
        bessel_i01(t, &i0, &i1);
        const double q = 0.25 * t * t;
        double a = 1.0, b = 1.0, hk = 0.0, s0 = 0.0, s1 = 0.0;
        s1 = (-gamma + (-gamma + 1.0)) * b;                 // k = 0: psi(1) + psi(2)
        for (int k = 1; k < 60; ++k) {
            a *= q / ((double)k * k);
            b *= q / ((double)k * (k + 1));
            hk += 1.0 / k;
            s0 += a * hk;
            s1 += b * ((-gamma + hk) + (-gamma + hk + 1.0 / (k + 1)));
        }
        *k0 = -(std::log(0.5 * t) + gamma) * i0 + s0;
        *k1 = 1.0 / t + std::log(0.5 * t) * i1 - 0.25 * t * s1;
        return;
    }
    // K_nu(t) = int_0^inf exp(-t cosh u) cosh(nu u) du: trapezoid, spectrally accurate
    const double h = 0.05;
    double a0 = 0.5 * std::exp(-t), a1 = a0;
    for (int j = 1;; ++j) {
        const double u = j * h, e = std::exp(-t * std::cosh(u));
        a0 += e;
        a1 += e * std::cosh(u);
        if (e < 1e-300 || e * std::cosh(u) < 1e-18 * a1) break;
    }
    *k0 = a0 * h;
    *k1 = a1 * h;
}

// F_s and its density dF/drho at rho, with the row constants c = K0(s)/I0(s) and
// den = 1 - 1/I0(s) precomputed.
struct ScreenedRow {
    double s = 0.0, c = 0.0, den = 1.0;
    explicit ScreenedRow(double s_) : s(s_) {
        if (s <= 0.0) return;
        double k0s, k1s, i0s, i1s;
        bessel_k01(s, &k0s, &k1s);
        bessel_i01(s, &i0s, &i1s);
        c = k0s / i0s;
        den = 1.0 - 1.0 / i0s;
    }
    void eval(double rho, double* F, double* p) const {
        if (!(rho > 0.0)) { *F = 0.0; *p = 0.0; return; }
        if (s <= 0.0) {
            const double l = -std::log(rho);
            *F = rho * rho * (1.0 + 2.0 * l);
            *p = 4.0 * rho * l;
            return;
        }
        const double t = rho * s;
        double k0t, k1t, i0t, i1t;
        bessel_k01(t, &k0t, &k1t);
        bessel_i01(t, &i0t, &i1t);
        *F = (1.0 - t * k1t - c * t * i1t) / den;
        *p = s * t * (k0t - c * i0t) / den;
    }
};

double screened_fixed_cdf(double rho, double s) {
    if (!(rho > 0.0)) return 0.0;
    if (rho >= 1.0) return 1.0;
    double F, p;
    ScreenedRow(s).eval(rho, &F, &p);
    return std::min(1.0, std::max(0.0, F));
}

double screened_fixed_node_u(int i, int cols) {
    const double v = (double)i / (double)(cols - 1);
    return v < 0.5 ? 2.0 * v * v : 1.0 - 2.0 * (1.0 - v) * (1.0 - v);
}

void screened_fixed_nodes(float* out, int rows, int cols, double xmax) {
    parallel_for(rows, [&](int j) {
        const ScreenedRow row_law(j == 0 ? 0.0 : std::expm1(xmax * (double)j / (double)(rows - 1)));
        float* row = out + (size_t)j * cols;
        row[0] = 0.0f;
        row[cols - 1] = 1.0f;
        double lo0 = 0.0, x = 0.5;   // targets increase along the row: brackets and guesses carry over
        for (int i = 1; i < cols - 1; ++i) {
            const double u = screened_fixed_node_u(i, cols);
            double lo = lo0, hi = 1.0;
            x = std::min(std::max(x, lo), hi);
            if (!(x > lo && x < hi)) x = 0.5 * (lo + hi);
            // safeguarded Newton: a step that leaves the bracket is replaced by bisection
            for (int it = 0; it < 100; ++it) {
                double F, p;
                row_law.eval(x, &F, &p);
                if (F < u) lo = x; else hi = x;
                const double xn = p > 0.0 ? x - (F - u) / p : -1.0;
                const double next = (xn > lo && xn < hi) ? xn : 0.5 * (lo + hi);
                if (std::fabs(next - x) <= 1e-15 * x || hi - lo <= 1e-16) { x = next; break; }
                x = next;
            }
            lo0 = lo;
            row[i] = (float)x;
        }
    }, 1);
}

}  // namespace wost
