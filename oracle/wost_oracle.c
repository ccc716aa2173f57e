/*
 * wost_oracle.c -- TEST INFRASTRUCTURE ONLY (see wost_oracle.h).
 *
 * CPU restatement of the reference's Walk-on-Stars path. Every function
 * cites the reference file:line it restates. Built with -ffp-contract=off so
 * that float32 expressions round like the reference's separate torch ops.
 */
#include "wost_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_PI 3.14159265358979323846
#define ORC_TABLE_N 4097

int orc_version(void) { return 1; }

/* ------------------------------------------------------------------------ */
/* Philox4x32-10 (Salmon et al. 2011); counter {step, 0, wid_lo, wid_hi}.    */
/* ------------------------------------------------------------------------ */
void orc_philox(uint32_t ctr[4], uint32_t k0, uint32_t k1, uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static float orc_u01(uint32_t v) { return (float)(v >> 8) * (1.0f / 16777216.0f); }

/* Relative perturbation of the step direction (0 = off). Used only by the
 * sensitivity test that measures how chaotic each scenario's walks are under
 * an ulp-sized change (tests/test_oracle_golden.py). */
static float orc_dir_perturb = 0.0f;
void orc_set_direction_perturbation(float rel) { orc_dir_perturb = rel; }

/* ------------------------------------------------------------------------ */
/* Geometry: geometry/PolylinesSimple.py                                      */
/* ------------------------------------------------------------------------ */

/* distance_to_polyline_jit :25-49 (NaN from a zero-length segment propagates) */
float orc_distance(const float* xy, int32_t nv, float px, float py) {
    float best = INFINITY;
    int isnan_ = 0;
    for (int i = 0; i + 1 < nv; ++i) {
        float ax = xy[2 * i], ay = xy[2 * i + 1], bx = xy[2 * i + 2], by = xy[2 * i + 3];
        float ux = bx - ax, uy = by - ay;                 /* :37 */
        float vx = px - ax, vy = py - ay;                 /* :38 */
        float duv = vx * ux + vy * uy;                    /* :41 */
        float duu = ux * ux + uy * uy;                    /* :42 */
        float t = duv / duu;                              /* :43 */
        if (t < 0.0f) t = 0.0f;
        if (t > 1.0f) t = 1.0f;
        float cx = (1.0f - t) * ax + t * bx;              /* :46 */
        float cy = (1.0f - t) * ay + t * by;
        float ex = cx - px, ey = cy - py;
        float d = sqrtf(ex * ex + ey * ey);               /* :47 */
        if (d != d) isnan_ = 1;
        if (d < best) best = d;                           /* :49 */
    }
    return isnan_ ? NAN : best;
}

/* is_silhouette_jit :51-81 */
static int orc_sil(const float* a, const float* b, const float* c, float px, float py) {
    float abx = b[0] - a[0], aby = b[1] - a[1];
    float bcx = c[0] - b[0], bcy = c[1] - b[1];
    float apx = px - a[0], apy = py - a[1];
    float bpx = px - b[0], bpy = py - b[1];
    float c1 = abx * apy - aby * apx;
    float c2 = bcx * bpy - bcy * bpx;
    return c1 * c2 < 0.0f;
}

void orc_is_silhouette(const float* xy, int32_t nv, float px, float py, uint8_t* mask) {
    for (int j = 1; j + 1 < nv; ++j)
        mask[j - 1] = (uint8_t)orc_sil(xy + 2 * (j - 1), xy + 2 * j, xy + 2 * (j + 1), px, py);
}

/* silhouette_distance_jit :83-102 */
float orc_silhouette_distance(const float* xy, int32_t nv, float px, float py) {
    float best = INFINITY;
    for (int j = 1; j + 1 < nv; ++j) {
        if (orc_sil(xy + 2 * (j - 1), xy + 2 * j, xy + 2 * (j + 1), px, py)) {
            float ex = xy[2 * j] - px, ey = xy[2 * j + 1] - py;
            float d = sqrtf(ex * ex + ey * ey);
            if (d < best) best = d;
        }
    }
    return best;
}

/* ray_intersection_jit :104-132 -- the returned "time" is the segment
 * parameter s (quirk Q1) */
void orc_ray_intersection(const float* xy, int32_t nv, float px, float py, float dx, float dy, float* times) {
    for (int i = 0; i + 1 < nv; ++i) {
        float ax = xy[2 * i], ay = xy[2 * i + 1];
        float ux = xy[2 * i + 2] - ax, uy = xy[2 * i + 3] - ay;
        float wx = px - ax, wy = py - ay;
        float d = dx * uy - dy * ux;                      /* :123 */
        float s = (dx * wy - dy * wx) / d;                /* :124 */
        float t = (ux * wy - uy * wx) / d;                /* :125 */
        int valid = (s >= 0.0f) && (s <= 1.0f) && (t > 0.0f);
        times[i] = valid ? s : INFINITY;
    }
}

/* intersect_polylines_jit :134-197; out5 = x, y, nx, ny, found */
void orc_intersect_polylines(const float* xy, int32_t nv, float px, float py, float dx, float dy,
                             float r, float* out5) {
    float dn = sqrtf(dx * dx + dy * dy);                  /* :149 */
    if (dn < 1e-10f) {
        out5[0] = px; out5[1] = py; out5[2] = 1.0f; out5[3] = 0.0f; out5[4] = 0.0f;
        return;
    }
    float ux_ = dx / dn, uy_ = dy / dn;                   /* :156 */
    float qx = px + 1e-6f * ux_, qy = py + 1e-6f * uy_;   /* :159 */
    float best = INFINITY;
    int idx = -1;
    float tmp;
    for (int i = 0; i + 1 < nv; ++i) {
        orc_ray_intersection(xy + 2 * i, 2, qx, qy, ux_, uy_, &tmp);
        if (isfinite(tmp) && (idx < 0 || tmp < best)) { best = tmp; idx = i; }
    }
    if (idx < 0 || best > r || best <= 0.0f) {            /* :166-174 */
        out5[0] = px + r * ux_; out5[1] = py + r * uy_;
        out5[2] = 0.0f; out5[3] = 0.0f; out5[4] = 0.0f;
        return;
    }
    float sx = xy[2 * idx + 2] - xy[2 * idx], sy = xy[2 * idx + 3] - xy[2 * idx + 1];
    float len = sqrtf(sx * sx + sy * sy);                 /* :184 */
    if (len < 1e-10f) {
        out5[2] = 0.0f; out5[3] = 1.0f;
    } else {
        float ex = sx / len, ey = sy / len;
        out5[2] = -ey; out5[3] = ex;                      /* :192-194 */
    }
    out5[0] = qx + best * ux_;                            /* :196 */
    out5[1] = qy + best * uy_;
    out5[4] = 1.0f;
}

/* ------------------------------------------------------------------------ */
/* Bessel functions (scipy.special i0/k0 as called at solvers/utils.py:21-24,43) */
/* ------------------------------------------------------------------------ */
double orc_i0(double x) {
    x = fabs(x);
    if (x <= 30.0) {
        double q = 0.25 * x * x, term = 1.0, s = 1.0;
        for (int k = 1; k < 200; ++k) {
            term *= q / ((double)k * (double)k);
            s += term;
            if (term < 1e-18 * s) break;
        }
        return s;
    }
    /* asymptotic: e^x / sqrt(2 pi x) * sum ((2k-1)!!)^2 / (k! (8x)^k) */
    double s = 1.0, term = 1.0;
    for (int k = 1; k < 30; ++k) {
        double nt = term * (2.0 * k - 1.0) * (2.0 * k - 1.0) / (8.0 * k * x);
        if (nt < 1e-18) break;
        term = nt;
        s += term;
    }
    return exp(x) / sqrt(2.0 * ORC_PI * x) * s;
}

double orc_k0(double x) {
    if (x <= 0.0) return INFINITY;
    if (x <= 2.0) {
        const double gamma = 0.57721566490153286061;
        double q = 0.25 * x * x, term = 1.0, i0 = 1.0, s = 0.0, h = 0.0;
        for (int k = 1; k < 60; ++k) {
            term *= q / ((double)k * (double)k);
            h += 1.0 / k;
            i0 += term;
            s += term * h;
        }
        return -(log(0.5 * x) + gamma) * i0 + s;
    }
    /* K0(x) = int_0^inf exp(-x cosh t) dt, composite Simpson */
    double h = 0.01, tmax = acosh(50.0 / x + 1.0) + 1.0;
    int n = (int)(tmax / h);
    if (n % 2) ++n;
    double s = exp(-x) + exp(-x * cosh(n * h));
    for (int j = 1; j < n; ++j) s += (j % 2 ? 4.0 : 2.0) * exp(-x * cosh(j * h));
    return s * h / 3.0;
}

/* screenedGreensNorm2D :29-44 */
double orc_screened_norm(double R, double sigma_bar) {
    double I = orc_i0(R * sqrt(sigma_bar));
    return 1.0 / sigma_bar * (1.0 - 1.0 / I);
}

/* ------------------------------------------------------------------------ */
/* Radial samplers as inverse CDFs of the rejection samplers' densities.     */
/*   GreensDistribution2D._refill_cache   solvers/utils.py:138-151           */
/*   ScreenedGreensDistribution2D._refill_cache :181-195                     */
/* node i = F^-1(i/(n-1)); a sample is the linear interpolation at u.        */
/* ------------------------------------------------------------------------ */
typedef struct { double s, kr_over_ir, M; } orc_sdens;

static double orc_screened_density(const orc_sdens* d, double rho) {
    double g = fabs((orc_k0(rho * d->s) - d->kr_over_ir * orc_i0(rho * d->s)) / (2.0 * ORC_PI));
    return g < d->M ? g : d->M;   /* accept w.p. min(g/M, 1)  (:193) */
}

void orc_sampler_nodes(int32_t screened, double sigma_bar, float* out, int32_t n) {
    const double a = 1e-6;
    if (!screened) {
        /* density -log(rho) on [a,1): F(rho) = (rho - rho log rho - c0) / z */
        double c0 = a - a * log(a), z = 1.0 - c0;
        for (int i = 0; i < n; ++i) {
            double u = (double)i / (double)(n - 1);
            if (i == 0) { out[i] = (float)a; continue; }
            if (i == n - 1) { out[i] = 1.0f; continue; }
            /* Newton from a bracketing bisection start */
            double lo = a, hi = 1.0, x = 0.5;
            for (int it = 0; it < 80; ++it) {
                x = 0.5 * (lo + hi);
                double F = (x - x * log(x) - c0) / z;
                if (F < u) lo = x; else hi = x;
            }
            for (int it = 0; it < 3; ++it) {
                double F = (x - x * log(x) - c0) / z, dF = -log(x) / z;
                if (dF > 0) x -= (F - u) / dF;
            }
            out[i] = (float)x;
        }
        return;
    }
    orc_sdens d;
    d.s = sqrt(sigma_bar);
    d.kr_over_ir = orc_k0(d.s) / orc_i0(d.s);
    d.M = orc_screened_norm(1.0, sigma_bar);
    const int J = 1 << 15;
    const double h = (1.0 - a) / J;
    double* C = (double*)malloc(sizeof(double) * (J + 1));
    double* p = (double*)malloc(sizeof(double) * (J + 1));
    for (int j = 0; j <= J; ++j) p[j] = orc_screened_density(&d, a + j * h);
    C[0] = 0.0;
    for (int j = 0; j < J; ++j) {
        double pm = orc_screened_density(&d, a + (j + 0.5) * h);
        C[j + 1] = C[j] + h / 6.0 * (p[j] + 4.0 * pm + p[j + 1]);
    }
    for (int i = 0; i < n; ++i) {
        if (i == 0) { out[i] = (float)a; continue; }
        if (i == n - 1) { out[i] = 1.0f; continue; }
        double T = C[J] * (double)i / (double)(n - 1);
        int lo = 0, hi = J;
        while (hi - lo > 1) {
            int mid = (lo + hi) / 2;
            if (C[mid] <= T) lo = mid; else hi = mid;
        }
        double x0 = a + lo * h, x = x0 + h * (T - C[lo]) / (C[lo + 1] - C[lo]);
        for (int it = 0; it < 4; ++it) {
            double xm = 0.5 * (x0 + x);
            double part = (x - x0) / 6.0 * (p[lo] + 4.0 * orc_screened_density(&d, xm) + orc_screened_density(&d, x));
            double px = orc_screened_density(&d, x);
            if (px > 0) x -= (C[lo] + part - T) / px;
        }
        out[i] = (float)x;
    }
    free(C);
    free(p);
}

static float orc_sample(const float* tab, float u) {
    float pos = u * (float)(ORC_TABLE_N - 1);
    int i = (int)pos;
    if (i > ORC_TABLE_N - 2) i = ORC_TABLE_N - 2;
    float f = pos - (float)i;
    return tab[i] + f * (tab[i + 1] - tab[i]);
}

/* ------------------------------------------------------------------------ */
/* Fields in double precision with value, gradient and Laplacian.            */
/* ------------------------------------------------------------------------ */
typedef struct { double v, gx, gy, l; } orc_jet;

static double sigm(double z) { return 1.0 / (1.0 + exp(-z)); }

/* Catmull-Rom spline as a cubic Hermite segment between nodes 1 and 2 with
 * tangents (P2-P0)/2 and (P3-P1)/2: weights of P0..P3 at t and their first
 * and second t-derivatives. */
static void orc_cr_basis(double t, double w[4], double d[4], double s[4]) {
    double t2 = t * t, t3 = t2 * t;
    double h00 = 2 * t3 - 3 * t2 + 1, h10 = t3 - 2 * t2 + t, h01 = -2 * t3 + 3 * t2, h11 = t3 - t2;
    double d00 = 6 * t2 - 6 * t, d10 = 3 * t2 - 4 * t + 1, d01 = -6 * t2 + 6 * t, d11 = 3 * t2 - 2 * t;
    double s00 = 12 * t - 6, s10 = 6 * t - 4, s01 = -12 * t + 6, s11 = 6 * t - 2;
    w[0] = -0.5 * h10; w[1] = h00 - 0.5 * h11; w[2] = 0.5 * h10 + h01; w[3] = 0.5 * h11;
    d[0] = -0.5 * d10; d[1] = d00 - 0.5 * d11; d[2] = 0.5 * d10 + d01; d[3] = 0.5 * d11;
    s[0] = -0.5 * s10; s[1] = s00 - 0.5 * s11; s[2] = 0.5 * s10 + s01; s[3] = 0.5 * s11;
}

/* one axis of a tabulated factor: clamp to the grid (constant outside),
 * node indices (clamped) and the derivative scale (0 outside) */
static void orc_grid_axis(double x, double x0, double ih, int n, int idx[4], double w[4], double d[4],
                          double s[4]) {
    double u = ((double)(float)x - x0) * ih, top = n - 1;
    int inside = u >= 0.0 && u <= top;
    if (u != u) u = 0.0;
    if (u < 0.0) u = 0.0;
    if (u > top) u = top;
    int i = (int)floor(u);
    if (i > n - 2) i = n - 2;
    orc_cr_basis(u - i, w, d, s);
    for (int k = 0; k < 4; ++k) {
        int q = i - 1 + k;
        idx[k] = q < 0 ? 0 : (q > n - 1 ? n - 1 : q);
        d[k] *= inside ? ih : 0.0;
        s[k] *= inside ? ih * ih : 0.0;
    }
}

static orc_jet orc_grid_jet(const orc_factor* f, const float* grid, double x, double y) {
    const float* p = f->p;
    int nx = (int)p[4], ny = (int)p[5];
    const float* g = grid + (int64_t)p[6];
    int ix[4], iy[4];
    double wx[4], dx[4], sx[4], wy[4], dy[4], sy[4];
    orc_grid_axis(x, p[0], p[2], nx, ix, wx, dx, sx);
    orc_grid_axis(y, p[1], p[3], ny, iy, wy, dy, sy);
    orc_jet j = {0, 0, 0, 0};
    for (int b = 0; b < 4; ++b) {
        double rv = 0, rd = 0, rs = 0;
        for (int a = 0; a < 4; ++a) {
            double v = g[(int64_t)iy[b] * nx + ix[a]];
            rv += wx[a] * v; rd += dx[a] * v; rs += sx[a] * v;
        }
        j.v += wy[b] * rv; j.gx += wy[b] * rd; j.gy += dy[b] * rv; j.l += wy[b] * rs + sy[b] * rv;
    }
    return j;
}

static orc_jet orc_factor_jet(const orc_factor* f, const float* grid, double x, double y) {
    const float* p = f->p;
    orc_jet j = {0, 0, 0, 0};
    switch (f->kind) {
    case 1: { /* x^a y^b */
        int a = (int)p[0], b = (int)p[1];
        double xa = pow(x, a), yb = pow(y, b);
        j.v = xa * yb;
        j.gx = a ? a * pow(x, a - 1) * yb : 0.0;
        j.gy = b ? b * xa * pow(y, b - 1) : 0.0;
        j.l = (a >= 2 ? a * (a - 1) * pow(x, a - 2) * yb : 0.0) + (b >= 2 ? b * (b - 1) * xa * pow(y, b - 2) : 0.0);
        break;
    }
    case 2: { /* exp of a quadratic in (x-cx, y-cy) */
        double dx = x - p[0], dy = y - p[1];
        double q = p[2] * dx * dx + p[3] * dy * dy + p[4] * dx * dy + p[5] * dx + p[6] * dy + p[7];
        double qx = 2.0 * p[2] * dx + p[4] * dy + p[5], qy = 2.0 * p[3] * dy + p[4] * dx + p[6];
        double e = exp(q);
        j.v = e; j.gx = e * qx; j.gy = e * qy; j.l = e * (qx * qx + qy * qy + 2.0 * p[2] + 2.0 * p[3]);
        break;
    }
    case 3: case 4: { /* sin / cos of a linear form */
        double l = (double)p[0] * x + (double)p[1] * y + p[2], aa = (double)p[0] * p[0] + (double)p[1] * p[1];
        double s = sin(l), c = cos(l);
        if (f->kind == 3) { j.v = s; j.gx = c * p[0]; j.gy = c * p[1]; j.l = -s * aa; }
        else { j.v = c; j.gx = -s * p[0]; j.gy = -s * p[1]; j.l = -c * aa; }
        break;
    }
    case 5: { /* sigmoid of a linear form */
        double s = sigm((double)p[0] * x + (double)p[1] * y + p[2]);
        double d1 = s * (1 - s), d2 = d1 * (1 - 2 * s);
        j.v = s; j.gx = d1 * p[0]; j.gy = d1 * p[1]; j.l = d2 * ((double)p[0] * p[0] + (double)p[1] * p[1]);
        break;
    }
    case 6: { /* utils.py:123-129: sigmoid(k (||x - c|| - R)) */
        double dx = x - p[1], dy = y - p[2], r = sqrt(dx * dx + dy * dy), k = p[0];
        double s = sigm(k * (r - p[3])), d1 = s * (1 - s), d2 = d1 * (1 - 2 * s);
        j.v = s; j.gx = d1 * k * dx / r; j.gy = d1 * k * dy / r; j.l = d2 * k * k + d1 * k / r;
        break;
    }
    case 7:
        j.v = ((float)x >= p[0] && (float)x <= p[1] && (float)y >= p[2] && (float)y <= p[3]) ? 1.0 : 0.0;
        break;
    case 8: {
        float dx = (float)x - p[0], dy = (float)y - p[1];
        j.v = (dx * dx + dy * dy <= p[2]) ? 1.0 : 0.0;
        break;
    }
    case 9: /* tabulated (Catmull-Rom bicubic) */
        if (!grid) { j.v = NAN; break; }
        j = orc_grid_jet(f, grid, x, y);
        break;
    default:
        j.v = NAN;
    }
    return j;
}

static orc_jet orc_field_jet(const orc_field* f, double x, double y) {
    orc_jet acc = {0, 0, 0, 0};
    if (!f) return acc;
    for (int t = 0; t < f->n_terms; ++t) {
        const orc_term* tm = &f->terms[t];
        orc_jet pr = {tm->coef, 0, 0, 0};
        for (int k = 0; k < tm->n_factors; ++k) {
            orc_jet q = orc_factor_jet(&f->factors[tm->first_factor + k], f->grid, x, y);
            orc_jet r;
            r.v = pr.v * q.v;
            r.gx = pr.v * q.gx + q.v * pr.gx;
            r.gy = pr.v * q.gy + q.v * pr.gy;
            r.l = pr.v * q.l + q.v * pr.l + 2.0 * (pr.gx * q.gx + pr.gy * q.gy);
            pr = r;
        }
        acc.v += pr.v; acc.gx += pr.gx; acc.gy += pr.gy; acc.l += pr.l;
    }
    return acc;
}

float orc_field_value(const orc_field* f, float x, float y) {
    if (!f) return 0.0f;
    return (float)orc_field_jet(f, x, y).v;
}

/* alpha and sigma with the defaults of solvers/WoStSolver.py:54-58 */
static orc_jet orc_alpha(const orc_problem* pb, float x, float y, int* detached) {
    if (!pb->alpha) {
        orc_jet one = {1.0, 0, 0, 0};
        *detached = 1;
        return one;
    }
    *detached = pb->alpha->flags & 1;
    return orc_field_jet(pb->alpha, x, y);
}

/* sigma_prime, solvers/WoStSolver.py:88-127 with torchLaplacian's +1e-8
 * (utils.py:54) and the clamp of alpha_wrapped (:80-86). */
float orc_sigma_prime(const orc_problem* pb, float x, float y) {
    int detached;
    orc_jet a = orc_alpha(pb, x, y, &detached);
    float av = (float)a.v;
    float ac = av < 1e-8f ? 1e-8f : av;
    float sg = pb->sigma ? orc_field_value(pb->sigma, x, y) : 0.0f;
    float ratio = sg / ac;                                   /* :102 */
    if (detached) return ratio;                              /* :123-127 (Q9) */
    int clamped = !(av >= 1e-8f);
    double gx = clamped ? 0.0 : a.gx, gy = clamped ? 0.0 : a.gy, lap = clamped ? 0.0 : a.l;
    double lapl = 1e-8 + lap;                                /* utils.py:54-59 */
    double lx = gx / ((double)ac + 1e-8), ly = gy / ((double)ac + 1e-8);   /* :108-114 */
    double gn = lx * lx + ly * ly;                           /* :115 */
    double corr = 0.5 * (lapl / ac - gn / 2.0);              /* :119 */
    return (float)((double)ratio + corr);
}

/* gridSampleMinMax(sigma_prime, bbox, 50) and the fallback of :130-136 */
double orc_sigma_bar(const orc_problem* pb) {
    float xmin = INFINITY, xmax = -INFINITY, ymin = INFINITY, ymax = -INFINITY;
    const float* arrs[2] = {pb->dxy, pb->nxy};
    int ns[2] = {pb->nd, pb->nn};
    for (int a = 0; a < 2; ++a)
        for (int i = 0; i < ns[a]; ++i) {
            float x = arrs[a][2 * i], y = arrs[a][2 * i + 1];
            if (x < xmin) xmin = x;
            if (x > xmax) xmax = x;
            if (y < ymin) ymin = y;
            if (y > ymax) ymax = y;
        }
    /* torch.linspace in float32 (counts up to the middle, down after) */
    float gx[50], gy[50];
    float sx = (xmax - xmin) / 49.0f, sy = (ymax - ymin) / 49.0f;
    for (int i = 0; i < 50; ++i) {
        gx[i] = i < 25 ? xmin + sx * (float)i : xmax - sx * (float)(49 - i);
        gy[i] = i < 25 ? ymin + sy * (float)i : ymax - sy * (float)(49 - i);
    }
    int any = 0;
    double lo = INFINITY, hi = -INFINITY;
    for (int i = 0; i < 50; ++i)
        for (int j = 0; j < 50; ++j) {
            float v = orc_sigma_prime(pb, gx[i], gy[j]);
            if (isnan(v) || isinf(v)) continue;
            any = 1;
            if (v < lo) lo = v;
            if (v > hi) hi = v;
        }
    if (!any) return NAN;
    double sb = hi - lo;
    if (sb <= 0.0 || sb > 1e3) sb = 10.0;
    return sb;
}

/* ------------------------------------------------------------------------ */
/* The walk: solvers/WoStSolver.py:187-298 for one walk.                     */
/* ------------------------------------------------------------------------ */
typedef struct {
    const orc_problem* pb;
    int delta, src, neu;
    float sigma_bar, sqrt_sb, inv_sb, rmin, eps;
    int max_steps;
    uint32_t k0, k1;
    const float* tab;
} orc_ctx;

static float orc_alpha_value(const orc_ctx* c, float x, float y) {
    int det;
    return (float)orc_alpha(c->pb, x, y, &det).v;
}

static float orc_gnorm(const orc_ctx* c, float r) {
    /* screenedGreensNorm2D(r, sigma_bar): R*sqrt(sigma_bar) in float32 */
    float xf = r * c->sqrt_sb;
    double I = orc_i0((double)xf);
    float inv = (float)(1.0 / I);
    return c->inv_sb * (1.0f - inv);
}

/* rec (may be NULL): the walk's history as return_history records it (:218-266), 4 floats
   per step: the pre-step point (path 'point') and the source sample point after the clip
   (contributions 'point'; the ray's point without a source), max_steps records. */
static void orc_walk(const orc_ctx* c, uint64_t wid, float x0, float y0, float* value, uint32_t* steps,
                     float* rec) {
    const orc_problem* pb = c->pb;
    float px = x0, py = y0;
    int k = 0;
    float dD = 1.0f;                                 /* :190 */
    int onB = 0;
    float nx = 0.0f, ny = 1.0f;                      /* :194 */
    float w = 1.0f;                                  /* :195 */
    float total = 0.0f;
    while (k < c->max_steps && dD > c->eps) {        /* :206 */
        dD = orc_distance(pb->dxy, pb->nd, px, py);  /* :208 */
        float r;
        if (c->neu) {
            float dn = orc_silhouette_distance(pb->nxy, pb->nn, px, py);
            float m = dn < dD ? dn : dD;             /* min(dD, dN) */
            r = m > c->rmin ? m : c->rmin;           /* max(rmin, .) :212 */
        } else {
            r = dD > c->rmin ? dD : c->rmin;         /* :215 */
        }
        uint32_t ctr[4] = {(uint32_t)k, 0u, (uint32_t)wid, (uint32_t)(wid >> 32)}, rn[4];
        orc_philox(ctr, c->k0, c->k1, rn);
        float theta = (orc_u01(rn[0]) * 2.0f) * (float)ORC_PI;      /* :226 */
        if (onB && c->neu) theta = theta / 2.0f + atan2f(ny, nx);    /* :227-228 */
        /* :230-232, the exact values rounded to float32 (torch's MKL cos/sin within
           its own ulp; the device's sincos_rn gives the same bits, tests/test_trig_rn.py) */
        float cs = (float)cos((double)theta), sn = (float)sin((double)theta);
        if (orc_dir_perturb != 0.0f) { cs *= 1.0f + orc_dir_perturb; sn *= 1.0f - orc_dir_perturb; }
        float xnx, xny;
        if (c->neu) {                                                /* :236 */
            float o[5];
            orc_intersect_polylines(pb->nxy, pb->nn, px, py, cs, sn, r, o);
            xnx = o[0]; xny = o[1]; nx = o[2]; ny = o[3]; onB = o[4] != 0.0f;
        } else {                                                     /* :238-239 */
            xnx = px + r * cs;
            xny = py + r * sn;
            onB = 0;
        }
        float yx = xnx, yy = xny, gn = 0.0f;
        if (c->src) {                                                /* :242-258 */
            float rs = orc_sample(c->tab, orc_u01(rn[1])) * r;       /* :244 */
            yx = px + rs * cs;                                       /* :245 */
            yy = py + rs * sn;
            float e1x = yx - px, e1y = yy - py, e2x = xnx - px, e2y = xny - py;
            float contrib;
            if (sqrtf(e1x * e1x + e1y * e1y) > sqrtf(e2x * e2x + e2y * e2y)) {   /* :248 */
                yx = xnx; yy = xny;
                contrib = 0.0f;
            } else if (c->delta) {                                   /* :252-254 */
                float f = orc_field_value(pb->f, yx, yy);
                gn = orc_gnorm(c, r);
                float ay = orc_alpha_value(c, yx, yy), ax = orc_alpha_value(c, px, py);
                contrib = ((f * gn) / sqrtf(ay * ax)) * w;
            } else {                                                 /* :256 */
                float f = orc_field_value(pb->f, yx, yy);
                contrib = f * ((r * r) / 4.0f);
            }
            total = total + contrib;                                 /* :258 */
        }
        if (rec) {                                                   /* :218-222, :261-266 */
            rec[4 * k + 0] = px; rec[4 * k + 1] = py;
            rec[4 * k + 2] = yx; rec[4 * k + 3] = yy;
        }
        if (c->delta) {                                              /* :271-284 */
            float mu = orc_u01(rn[2]);
            gn = orc_gnorm(c, r);                                    /* :273 */
            float ax = orc_alpha_value(c, px, py);
            if (mu > c->sigma_bar * gn) {
                float an = orc_alpha_value(c, xnx, xny);
                w = w * sqrtf(an / ax);                              /* :277 */
                px = xnx; py = xny;
            } else {
                float spv = orc_sigma_prime(pb, yx, yy);             /* :281 */
                float sc = 1.0f - spv / c->sigma_bar;
                if (0.0f > sc) sc = 0.0f;                            /* :282 */
                float ay = orc_alpha_value(c, yx, yy);
                w = (w * sqrtf(ay / ax)) * sc;                       /* :283 */
                px = yx; py = yy;
            }
        } else {
            px = xnx; py = xny;                                      /* :287 */
        }
        k += 1;                                                      /* :291 */
    }
    float g = orc_field_value(pb->g, px, py);                        /* :295 */
    if (c->delta) g = g * w;                                         /* :296-297 */
    total = total + g;
    *value = total;
    *steps = (uint32_t)k;
}

/* records (may be NULL): [wid_end - wid_begin][max_steps][4] floats of orc_walk's rec */
int orc_solve_history(const orc_problem* pb, const float* points, int64_t n_points, int64_t W,
                      int64_t wid_begin, int64_t wid_end, int32_t max_steps, float eps, uint64_t seed,
                      int32_t threads, float* walk_values, uint32_t* walk_steps, float* records) {
    if (!pb || !pb->dxy || pb->nd < 2 || W <= 0 || wid_begin < 0 || wid_end < wid_begin ||
        wid_end > n_points * W)
        return -1;
    orc_ctx c;
    memset(&c, 0, sizeof(c));
    c.pb = pb;
    c.delta = pb->sigma != NULL || pb->alpha != NULL;
    c.src = pb->f != NULL;
    c.neu = pb->nxy != NULL && pb->nn > 0;
    if (c.delta && !c.src) return -2;   /* the reference raises UnboundLocalError (:281) */
    double sb = 0.0;
    if (c.delta) sb = pb->sigma_bar > 0.0 ? pb->sigma_bar : orc_sigma_bar(pb);
    c.sigma_bar = (float)sb;
    c.sqrt_sb = (float)sqrt(sb);
    c.inv_sb = sb > 0 ? (float)(1.0 / sb) : 0.0f;
    c.rmin = eps / 2.0f;
    c.eps = eps;
    c.max_steps = max_steps;
    c.k0 = (uint32_t)seed;
    c.k1 = (uint32_t)(seed >> 32);
    /* sampler nodes, cached across calls (building the screened table costs ~1 s) */
    static float tab_cache[ORC_TABLE_N];
    static int cache_kind = -1;
    static double cache_sb = -1.0;
    if (c.src) {
        if (cache_kind != c.delta || cache_sb != sb) {
            orc_sampler_nodes(c.delta, sb, tab_cache, ORC_TABLE_N);
            cache_kind = c.delta;
            cache_sb = sb;
        }
    }
    c.tab = tab_cache;
    int64_t n = wid_end - wid_begin;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t i = 0; i < n; ++i) {
        uint64_t wid = (uint64_t)(wid_begin + i);
        int64_t p = (int64_t)(wid / (uint64_t)W);
        orc_walk(&c, wid, points[2 * p], points[2 * p + 1], &walk_values[i], &walk_steps[i],
                 records ? records + (size_t)i * (size_t)max_steps * 4u : NULL);
    }
    return 0;
}

int orc_solve(const orc_problem* pb, const float* points, int64_t n_points, int64_t W,
              int64_t wid_begin, int64_t wid_end, int32_t max_steps, float eps, uint64_t seed,
              int32_t threads, float* walk_values, uint32_t* walk_steps) {
    return orc_solve_history(pb, points, n_points, W, wid_begin, wid_end, max_steps, eps, seed, threads,
                             walk_values, walk_steps, NULL);
}
