/*
 * wost_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, CPU restatement of the reference's Walk-on-Stars hot path
 * (Tsuchijo/DCRMonteCarlo, solvers/WoStSolver.py:162-316 and
 * geometry/PolylinesSimple.py:13-197). It is the parity checker for the HIP
 * kernels of libwost.so and the CPU baseline of bench.py (kind "port").
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it; the product (dcrmontecarlo_amd) never does.
 *
 * Pinned against the reference: tests/golden/ holds vectors produced by
 * running the reference itself in the build container
 * (tools/gen_fixtures.py) -- geometry KATs, sigma'/sigma_bar, Green's norms,
 * sampler draws and per-walk trajectories replayed on this oracle's Philox
 * stream.
 *
 * The oracle shares no source with libwost: it has its own Philox, its own
 * Bessel functions, its own sampler construction and its own field
 * evaluation (double precision). It takes fields in the same
 * sum-of-products encoding as include/wost.h (that encoding is the problem
 * description, not an implementation).
 */
#ifndef WOST_ORACLE_H
#define WOST_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { int32_t kind; float p[8]; } orc_factor;
typedef struct { float coef; int32_t first_factor; int32_t n_factors; } orc_term;
typedef struct {
    const orc_term* terms; int32_t n_terms;
    const orc_factor* factors; int32_t n_factors;
    int32_t flags;     /* 1 = alpha detached (sigma' = sigma/alpha) */
    const float* grid; int64_t n_grid;   /* kind-9 (tabulated) factor values */
} orc_field;

typedef struct {
    const float* dxy; int32_t nd;      /* Dirichlet vertices */
    const float* nxy; int32_t nn;      /* Neumann vertices (nn == 0: none) */
    const orc_field* g;                /* NULL: 0 */
    const orc_field* f;                /* NULL: no source */
    const orc_field* sigma;            /* NULL */
    const orc_field* alpha;            /* NULL */
    double sigma_bar;                  /* <= 0: estimate like the reference */
} orc_problem;

int orc_version(void);

/* geometry (PolylinesSimple.py) */
float orc_distance(const float* xy, int32_t nv, float px, float py);
float orc_silhouette_distance(const float* xy, int32_t nv, float px, float py);
void orc_is_silhouette(const float* xy, int32_t nv, float px, float py, uint8_t* mask);
void orc_ray_intersection(const float* xy, int32_t nv, float px, float py, float dx, float dy, float* times);
void orc_intersect_polylines(const float* xy, int32_t nv, float px, float py, float dx, float dy,
                             float r, float* out5);

/* Green's norms and samplers (solvers/utils.py) */
double orc_i0(double x);
double orc_k0(double x);
double orc_screened_norm(double R, double sigma_bar);
void orc_sampler_nodes(int32_t screened, double sigma_bar, float* out, int32_t n);

/* fields and sigma' (WoStSolver.py:66-138) */
float orc_field_value(const orc_field* f, float x, float y);
float orc_sigma_prime(const orc_problem* pb, float x, float y);
double orc_sigma_bar(const orc_problem* pb);

/* sensitivity probe: relative perturbation of the step direction (0 = off) */
void orc_set_direction_perturbation(float rel);

/* Philox4x32-10 */
void orc_philox(uint32_t ctr[4], uint32_t k0, uint32_t k1, uint32_t out[4]);

/* _solveUnified over global walks [wid_begin, wid_end) of points[n_points][2]
 * with walks_per_point W. Writes per-walk values and steps (walk order).
 * threads <= 0: OpenMP default. Returns 0 or a negative error. */
int orc_solve(const orc_problem* pb, const float* points, int64_t n_points, int64_t W,
              int64_t wid_begin, int64_t wid_end, int32_t max_steps, float eps, uint64_t seed,
              int32_t threads, float* walk_values, uint32_t* walk_steps);
/* orc_solve with return_history's records (:218-266): records[walk][max_steps][4] =
 * the pre-step point and the source sample point after the clip (the ray's point
 * without a source), for steps 0 .. walk_steps - 1 (records may be NULL). */
int orc_solve_history(const orc_problem* pb, const float* points, int64_t n_points, int64_t W,
                      int64_t wid_begin, int64_t wid_end, int32_t max_steps, float eps, uint64_t seed,
                      int32_t threads, float* walk_values, uint32_t* walk_steps, float* records);

#ifdef __cplusplus
}
#endif
#endif
