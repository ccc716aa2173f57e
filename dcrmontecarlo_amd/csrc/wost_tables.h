// wost_tables.h -- host-side numerics of libwost: modified Bessel functions in
// double precision, the Chebyshev fits of i0e used by the kernel, and the
// inverse-CDF nodes of the reference's radial samplers.
#pragma once

#include <vector>

namespace wost {

// i0e(x) = exp(-x) I0(x), x >= 0, ~1e-15 relative (trapezoid rule on the
// periodic integral (1/pi) int_0^pi exp(x (cos t - 1)) dt).
double i0e_host(double x);
// I0(x) (may overflow to inf for x > ~700).
double i0_host(double x);
// K0(x), x > 0 (series for x <= 2, trapezoid on int_0^inf exp(-x cosh t) dt otherwise).
double k0_host(double x);

// Chebyshev coefficients: ca[24] for i0e on [0,8] in t = x/4-1,
// cb[20] for sqrt(x) i0e(x) on (8,inf) in t = 16/x-1.
void fit_i0e_chebyshev(float* ca, int na, float* cb, int nb);

// screenedGreensNorm2D(R, sigma_bar) (solvers/utils.py:29-44), double.
double screened_greens_norm(double R, double sigma_bar);
// screenedGreens2D at distance r for ball radius R (solvers/utils.py:5-26), double.
double screened_greens(double r, double R, double sigma_bar);

// Cubic coefficients {a0, a1, a2, a3} per cell (4 floats each) of
// Phi(x) = (1 - 1/I0(x)) / x^2 on cells [c h, (c+1) h), h = xmax / cells,
// in t = x/h - c: Hermite interpolation of Phi and h Phi' at the cell ends,
// both from the power series of I0 and I1 in double (wost_device.h
// greens_norm_from_table).
void greens_norm_cells(float* out, int cells, double xmax);
// Phi(x) and Phi'(x) in double.
void greens_phi(double x, double* phi, double* dphi);

// Inverse-CDF nodes F^-1(i/(n-1)), i = 0..n-1, of
//  * GreensDistribution2D (solvers/utils.py:138-151): density -log(rho) on [1e-6, 1);
//  * ScreenedGreensDistribution2D (solvers/utils.py:181-195): density
//    min(|G_sigmabar(rho; R=1)|, screenedGreensNorm2D(1, sigma_bar)) on [1e-6, 1).
void greens_sampler_nodes(float* out, int n);
// compat="fixed" (quirk Q3 corrected): the radial density of a point sampled
// from the ball's Green's function in 2-D, rho ln(1/rho) on (0, 1) (the
// Jacobian rho included); F(rho) = rho^2 (1 + 2 ln(1/rho)).
void greens_sampler_nodes_jacobian(float* out, int n);
void screened_sampler_nodes(float* out, int n, double sigma_bar);

// compat="fixed" screened sampler (Q4/Q5 corrected): the exact radial law of a
// point sampled from the ball's screened Green's function, CDF F_s(rho) for the
// shape parameter s = R sqrt(sigma_bar) (closed form in I0, I1, K0, K1; s = 0: the
// Laplace law). screened_fixed_nodes fills [rows][cols] inverse-CDF nodes: row j
// is s_j = expm1(xmax j / (rows-1)) (row 0: s = 0), column i the quantile
// u_i = screened_fixed_node_u(i, cols) = 2 v^2 (v < 1/2) or 1 - 2 (1-v)^2, v =
// i / (cols-1), so that the steep ends of the inverse CDF are resolved
// (wost_device.h sample_rho_screened_fixed).
double screened_fixed_cdf(double rho, double s);
double screened_fixed_node_u(int i, int cols);
void screened_fixed_nodes(float* out, int rows, int cols, double xmax);

}  // namespace wost
