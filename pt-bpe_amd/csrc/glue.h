// Glue optimisation of the RMSD mode: L-BFGS over the glue angles
// of a whole chain, so that the NeRF of the quantized chain puts each residue's frame
// back on the exit frames cached from the chain before quantization.
//
//   reference                                         here
//   BPE.fk_segment_torch (ret_all)  bpe.py:423-459    glue_eval: NeRF forward + frames
//   optimize_glues_entry_torch      bpe.py:462-578    glue_eval (loss, prior, gradient by a
//     closure / circ_kde_prior                          hand-written reverse sweep) and
//   torch.optim.LBFGS(max_iter=20,                    k_glue_opt: the optimiser's control
//     line_search_fn="strong_wolfe")                  flow (torch/optim/lbfgs.py), restated
//   BPE._opt_glue_worker / opt_glue bpe.py:739-807    host: geobpe/glue.py
//
// One thread per chain (the chains are independent problems; the reference runs one
// process-pool task per chain).  Per-chain state lives in global memory interleaved over
// the chains (element i of chain s at i * S + s), so a wave's threads touch consecutive
// words while they step through their chains together.
//
// Arithmetic follows the reference's dtypes: parameters, gradients and the optimiser's
// vectors are float32 (the torch parameter is float32); the angles' sines and cosines and
// the placement offsets d are float32 (place_dihedral computes them on float32 tensors);
// atom positions, frames and the loss are float64 (the NeRF starts from float64 initial
// coordinates, nerf.py:88-89, so every later tensor is promoted).
#pragma once

#include "featurize.h"
#include "rmsd.h"

namespace gb {

constexpr int GLUE_HIST = 20;  // max_iter = 20: at most 19 (s, y) pairs are kept
constexpr int GLUE_NVEC = 9;   // float vectors per chain besides the history

struct GlueProb {
  int64_t S;            // chains in the batch (interleave stride)
  const int64_t* roff;  // residue offsets [S + 1]
  const double* geo;    // 9 per residue (float32-representable values), rmsd.h k_nerf layout
  const float* tgt;     // 12 per glue: exit frame R (row-major 3x3) and t, float32
  const int32_t* grid;  // per chain: index of its prior table
  const float* prior;   // per grid: 3 types x (centres[kmax], weights[kmax])
  const int32_t* kcnt;  // per grid: 3 bin counts
  int32_t kmax;
  float lam;
  double wR, wt;
  double* X;   // atoms, 9 per residue, interleaved
  double* AX;  // their adjoints
  float* V;    // GLUE_NVEC vectors of pmax, interleaved
  float* H;    // 2 * GLUE_HIST vectors of pmax (s and y), interleaved
  int64_t pmax;
};

// float32 elementary functions rounded from float64: the reference's float32 torch ops on
// the CPU (glibc / SLEEF, ~correctly rounded) are matched more closely than by the ~1-2 ulp
// single-precision device library, and the trajectory of 20 L-BFGS iterations amplifies
// every ulp
__device__ inline float f_sin(float a) { return (float)sin((double)a); }
__device__ inline float f_cos(float a) { return (float)cos((double)a); }
__device__ inline float f_atan2(float y, float x) { return (float)atan2((double)y, (double)x); }
__device__ inline float f_exp(float a) { return (float)exp((double)a); }
__device__ inline float f_log(float a) { return (float)log((double)a); }

struct IV {  // a strided float vector of one chain
  float* p;
  int64_t S;
  __device__ float& operator[](int64_t i) const { return p[i * S]; }
};

__device__ inline float glue_wrap(float a) {
  // torch.remainder(torch.atan2(sin a, cos a) + 2 pi, 2 pi) on float32 (bpe.py:490-493)
  const float two_pi = 6.28318530717958647692f;
  float w = f_atan2(f_sin(a), f_cos(a)) + two_pi;
  float r = fmodf(w, two_pi);
  if (r < 0.f) r += two_pi;
  return r;
}

// autograd of glue_wrap: remainder passes the gradient; atan2(y = sin a, x = cos a) gives
// g x / (y^2 + x^2) to y and -g y / (y^2 + x^2) to x; then sin' = cos, cos' = -sin
__device__ inline float glue_wrap_back(float a, float g) {
  const float y = f_sin(a), x = f_cos(a);
  const float den = y * y + x * x;
  return (g * x / den) * x + (g * -y / den) * (-y);
}

// the placement offsets (float32, place_dihedral's d before .type(m.dtype), nerf.py:200-207)
__device__ inline void glue_d(float A, float L, float T, float& d0, float& d1, float& d2) {
  const float cA = f_cos(A), sA = f_sin(A), cT = f_cos(T), sT = f_sin(T);
  d0 = -L * cA;
  d1 = L * cT * sA;
  d2 = L * sT * sA;
}

__device__ inline V3 v_addv(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }

__device__ inline V3 glue_place(V3 a, V3 b, V3 c, float A, float L, float T) {
  const V3 ab = v_sub(b, a);
  const V3 u = v_sub(c, b);
  const V3 bc = v_scale(u, 1.0 / v_norm(u));
  const V3 m = v_cross(ab, bc);
  const V3 n = v_scale(m, 1.0 / v_norm(m));
  const V3 nbc = v_cross(n, bc);
  float f0, f1, f2;
  glue_d(A, L, T, f0, f1, f2);
  const double d0 = f0, d1 = f1, d2 = f2;
  return {bc.x * d0 + nbc.x * d1 + n.x * d2 + c.x, bc.y * d0 + nbc.y * d1 + n.y * d2 + c.y,
          bc.z * d0 + nbc.z * d1 + n.z * d2 + c.z};
}

// reverse of glue_place: G = dL/d(out); adds to the adjoints of a, b, c and returns the
// float32 gradients of the angle A and torsion T
__device__ inline void glue_place_back(V3 a, V3 b, V3 c, float A, float L, float T, V3 G, V3& ga, V3& gb_, V3& gc,
                                       float& gA, float& gT) {
  const V3 ab = v_sub(b, a);
  const V3 u = v_sub(c, b);
  const double lu = v_norm(u);
  const V3 bc = v_scale(u, 1.0 / lu);
  const V3 m = v_cross(ab, bc);
  const double lm = v_norm(m);
  const V3 n = v_scale(m, 1.0 / lm);
  const V3 nbc = v_cross(n, bc);
  float f0, f1, f2;
  glue_d(A, L, T, f0, f1, f2);
  // d (float64 after the cast) -> the float32 gradient of d, then float32 chain rule
  const float g0 = (float)v_dot(G, bc), g1 = (float)v_dot(G, nbc), g2 = (float)v_dot(G, n);
  // autograd's float32 chain through d0 = (-L) cos A, d1 = (L cos T) sin A, d2 = (L sin T) sin A
  const float cA = f_cos(A), sA = f_sin(A), cT = f_cos(T), sT = f_sin(T);
  gA = ((g0 * (-L)) * (-sA) + (g1 * (L * cT)) * cA) + (g2 * (L * sT)) * cA;
  gT = ((g1 * sA) * L) * (-sT) + ((g2 * sA) * L) * cT;
  gc = v_addv(gc, G);
  V3 g_bc = v_scale(G, (double)f0);
  const V3 g_nbc = v_scale(G, (double)f1);
  V3 g_n = v_scale(G, (double)f2);
  g_n = v_addv(g_n, v_cross(bc, g_nbc));
  g_bc = v_addv(g_bc, v_cross(g_nbc, n));
  const V3 g_m = v_scale(v_sub(g_n, v_scale(n, v_dot(n, g_n))), 1.0 / lm);
  const V3 g_ab = v_cross(bc, g_m);
  g_bc = v_addv(g_bc, v_cross(g_m, ab));
  const V3 g_u = v_scale(v_sub(g_bc, v_scale(bc, v_dot(bc, g_bc))), 1.0 / lu);
  gc = v_addv(gc, g_u);
  gb_ = v_addv(v_sub(gb_, g_u), g_ab);
  ga = v_sub(ga, g_ab);
}

// _normalize(v, eps) = v / (|v| + eps) and its reverse (angles_and_coords.py:567-569)
__device__ inline V3 glue_normalize(V3 v) { return v_scale(v, 1.0 / (v_norm(v) + 1e-8)); }
__device__ inline V3 glue_normalize_back(V3 v, V3 g) {
  const double l = v_norm(v), s = l + 1e-8;
  return v_sub(v_scale(g, 1.0 / s), v_scale(v, v_dot(v, g) / (l * s * s)));
}

__device__ inline V3 ldx(const double* X, int64_t S, int64_t atom) {
  const double* p = X + atom * 3 * S;
  return {p[0], p[S], p[2 * S]};
}
__device__ inline void stx(double* X, int64_t S, int64_t atom, V3 v) {
  double* p = X + atom * 3 * S;
  p[0] = v.x;
  p[S] = v.y;
  p[2 * S] = v.z;
}

// loss and gradient of one chain at the parameters x (glue k = (omega_k, theta_k, phi_k),
// raw values; wrapped here as the closure does)
__device__ double glue_eval(const GlueProb& P, int64_t s, int64_t r, const double* g, const float* tg,
                            const float* pr, const int32_t* kc, IV x, IV grad) {
  const int64_t S = P.S;
  double* X = P.X + s;
  double* AX = P.AX + s;
  // -- forward: update_backbone_positions from the float32 values, then NeRF (nerf.py:85-128)
  V3 p3, p2, p1;
  backbone_start(g[1], g[0], g[2], p3, p2, p1);
  stx(X, S, 0, p3);
  stx(X, S, 1, p2);
  stx(X, S, 2, p1);
  for (int64_t k = 0; k + 1 < r; k++) {
    const double* gk = g + 9 * k;
    const double* gn = gk + 9;
    const float om = glue_wrap(x[3 * k]), th = glue_wrap(x[3 * k + 1]), ph = glue_wrap(x[3 * k + 2]);
    const V3 nN = glue_place(p3, p2, p1, (float)gk[4], (float)gk[3], (float)gk[6]);
    const V3 nCA = glue_place(p2, p1, nN, th, (float)gn[0], om);
    const V3 nC = glue_place(p1, nN, nCA, (float)gn[2], (float)gn[1], ph);
    stx(X, S, 3 * (k + 1), nN);
    stx(X, S, 3 * (k + 1) + 1, nCA);
    stx(X, S, 3 * (k + 1) + 2, nC);
    p3 = nN;
    p2 = nCA;
    p1 = nC;
  }
  for (int64_t a = 0; a < 3; a++) stx(AX, S, a, V3{0, 0, 0});  // atoms 3.. are written below
  // -- frames of residues 1..r-1 against the targets (bpe.py:539-548)
  double rot = 0.0, trans = 0.0;
  for (int64_t k = 0; k + 1 < r; k++) {
    const int64_t i = k + 1;
    const V3 N = ldx(X, S, 3 * i), CA = ldx(X, S, 3 * i + 1), C = ldx(X, S, 3 * i + 2);
    const float* T = tg + 12 * k;
    const V3 vx = v_sub(C, CA), vu = v_sub(N, CA);
    const V3 ex = glue_normalize(vx), eu = glue_normalize(vu);
    const V3 w = v_cross(ex, eu);
    const V3 ez = glue_normalize(w);
    const V3 ey = v_cross(ez, ex);
    const V3 Rx = {T[0], T[3], T[6]}, Ry = {T[1], T[4], T[7]}, Rz = {T[2], T[5], T[8]}, Rt = {T[9], T[10], T[11]};
    const V3 dx = v_sub(ex, Rx), dy = v_sub(ey, Ry), dz = v_sub(ez, Rz), dt = v_sub(CA, Rt);
    rot += 0.5 * (v_dot(dx, dx) + v_dot(dy, dy) + v_dot(dz, dz));
    trans += v_dot(dt, dt);
    V3 gx = v_scale(dx, P.wR), gy = v_scale(dy, P.wR), gz = v_scale(dz, P.wR);
    gz = v_addv(gz, v_cross(ex, gy));
    gx = v_addv(gx, v_cross(gy, ez));
    const V3 gw = glue_normalize_back(w, gz);
    gx = v_addv(gx, v_cross(eu, gw));
    const V3 gu = v_cross(gw, ex);
    const V3 gvx = glue_normalize_back(vx, gx), gvu = glue_normalize_back(vu, gu);
    stx(AX, S, 3 * i + 2, gvx);  // each atom's frame term, written once
    stx(AX, S, 3 * i, gvu);
    stx(AX, S, 3 * i + 1, v_addv(v_scale(v_addv(gvx, gvu), -1.0), v_scale(dt, 2.0 * P.wt)));
  }
  double loss = P.wR * rot + P.wt * trans;
  // -- prior: mixture of von Mises per glue angle (bpe.py:527-534, 549-558), float32
  float prior = 0.f;
  for (int64_t k = 0; k + 1 < r; k++) {
    float gp[3];
    float term = 0.f;
    for (int t = 0; t < 3; t++) {
      gp[t] = 0.f;
      if (P.lam == 0.f) continue;
      const float a = glue_wrap(x[3 * k + t]);
      const float kappa = t == 0 ? 50.f : 20.f;
      const float* cen = pr + (2 * t) * P.kmax;
      const float* wt = cen + P.kmax;
      float mx = -INFINITY;
      for (int j = 0; j < kc[t]; j++) mx = fmaxf(mx, kappa * f_cos(a - cen[j]) + f_log(wt[j] + 1e-12f));
      float se = 0.f, sg = 0.f;
      for (int j = 0; j < kc[t]; j++) {
        const float e = f_exp(kappa * f_cos(a - cen[j]) + f_log(wt[j] + 1e-12f) - mx);
        se += e;
        sg += e * kappa * f_sin(a - cen[j]);
      }
      term += -(mx + f_log(se));
      gp[t] = P.lam * (sg / se);
    }
    prior += term;
    grad[3 * k] = gp[0];
    grad[3 * k + 1] = gp[1];
    grad[3 * k + 2] = gp[2];
  }
  if (P.lam != 0.f) loss += (double)(P.lam * prior);
  // -- reverse sweep over the placements (atoms 3r-1 .. 3; atoms 0..2 hold no parameter).
  // Atom m's adjoint takes its frame term plus the placements of atoms m+1..m+3, so walking
  // down, the adjoints of j-1 and j-2 and the atoms j-1, j-2 ride in registers and each step
  // loads only atom j-3 and its frame term (no store-to-load round trip through memory)
  V3 R0 = ldx(AX, S, 3 * r - 1), R1 = ldx(AX, S, 3 * r - 2), R2 = ldx(AX, S, 3 * r - 3);
  V3 C1 = ldx(X, S, 3 * r - 2), C2 = ldx(X, S, 3 * r - 3);
  for (int64_t j = 3 * r - 1; j >= 3; j--) {
    const int64_t i = j / 3, k = i - 1;
    const double* gk = g + 9 * k;
    const double* gn = gk + 9;
    const V3 C3 = ldx(X, S, j - 3);
    V3 R3 = ldx(AX, S, j - 3);
    float gA = 0.f, gT = 0.f;
    if (j % 3 == 0) {
      glue_place_back(C3, C2, C1, (float)gk[4], (float)gk[3], (float)gk[6], R0, R3, R2, R1, gA, gT);
    } else if (j % 3 == 1) {
      const float om = glue_wrap(x[3 * k]), th = glue_wrap(x[3 * k + 1]);
      glue_place_back(C3, C2, C1, th, (float)gn[0], om, R0, R3, R2, R1, gA, gT);
      grad[3 * k] += gT;
      grad[3 * k + 1] += gA;
    } else {
      const float ph = glue_wrap(x[3 * k + 2]);
      glue_place_back(C3, C2, C1, (float)gn[2], (float)gn[1], ph, R0, R3, R2, R1, gA, gT);
      grad[3 * k + 2] += gT;
    }
    R0 = R1;
    R1 = R2;
    R2 = R3;
    C1 = C2;
    C2 = C3;
  }
  for (int64_t i = 0; i < 3 * (r - 1); i++) grad[i] = glue_wrap_back(x[i], grad[i]);
  return loss;
}

// _cubic_interpolate (torch/optim/lbfgs.py)
__device__ inline float glue_cubic(float x1, double f1, float g1, float x2, double f2, float g2, bool bounded,
                                   float lo, float hi) {
  float xmin = bounded ? lo : fminf(x1, x2), xmax = bounded ? hi : fmaxf(x1, x2);
  if (!bounded && !(x1 <= x2)) {
    xmin = x2;
    xmax = x1;
  }
  const float d1 = g1 + g2 - (float)(3.0 * (f1 - f2) / (double)(x1 - x2));
  const float d2s = d1 * d1 - g1 * g2;
  if (d2s >= 0.f) {
    const float d2 = sqrtf(d2s);
    float mp;
    if (x1 <= x2)
      mp = x2 - (x2 - x1) * ((g2 + d2 - d1) / (g2 - g1 + 2.f * d2));
    else
      mp = x1 - (x1 - x2) * ((g1 + d2 - d1) / (g1 - g2 + 2.f * d2));
    return fminf(fmaxf(mp, xmin), xmax);
  }
  return (xmin + xmax) / 2.f;
}

__device__ inline float glue_dot(IV a, IV b, int64_t n) {
  float s = 0.f;
  for (int64_t i = 0; i < n; i++) s += a[i] * b[i];
  return s;
}
__device__ inline void glue_copy(IV dst, IV src, int64_t n) {
  for (int64_t i = 0; i < n; i++) dst[i] = src[i];
}

__global__ __launch_bounds__(64) void k_glue_opt(GlueProb P, const float* x0, float* xout, int32_t* stats,
                                                 double* losses) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= P.S) return;
  const int64_t a0 = P.roff[s], r = P.roff[s + 1] - a0;
  const int64_t np = 3 * (r - 1), g0 = a0 - s;  // glues of this chain and their first index
  if (r < 2) {  // no glue
    stats[2 * s] = 0;
    stats[2 * s + 1] = 0;
    losses[2 * s] = 0.0;
    losses[2 * s + 1] = 0.0;
    return;
  }
  const double* g = P.geo + 9 * a0;
  const float* tg = P.tgt + 12 * g0;
  const int32_t gi = P.grid[s];
  const float* pr = P.prior + (int64_t)gi * 6 * P.kmax;
  const int32_t* kc = P.kcnt + 3 * gi;
  const int64_t S = P.S, PM = P.pmax;
  auto vec = [&](int v) { return IV{P.V + (int64_t)v * PM * S + s, S}; };
  auto hs = [&](int h) { return IV{P.H + (int64_t)h * PM * S + s, S}; };
  auto hy = [&](int h) { return IV{P.H + (int64_t)(GLUE_HIST + h) * PM * S + s, S}; };
  IV x = vec(0), d = vec(1), fg = vec(2), pg = vec(3), xi = vec(4), q = vec(5);
  int gb[3] = {6, 7, 8};  // line-search gradient buffers (g_new, g_prev / bracket)
  float ro[GLUE_HIST], al[GLUE_HIST];
  int nold = 0;
  for (int64_t i = 0; i < np; i++) x[i] = x0[3 * g0 + i];
  // evaluation at x_init + t d (LBFGS._directional_evaluate)
  auto eval_at = [&](float t, IV out) -> double {
    for (int64_t i = 0; i < np; i++) q[i] = xi[i] + t * d[i];
    return glue_eval(P, s, r, g, tg, pr, kc, q, out);
  };
  double loss = glue_eval(P, s, r, g, tg, pr, kc, x, fg);
  const double loss0 = loss;
  int evals = 1, n_iter = 0;
  float amax = 0.f;
  for (int64_t i = 0; i < np; i++) amax = fmaxf(amax, fabsf(fg[i]));
  const float tol_grad = 1e-7f, tol_change = 1e-9f;
  const int max_iter = 20, max_eval = 25;
  float t = 1.f, H_diag = 1.f;
  double prev_loss = loss;
  if (!(amax <= tol_grad)) {
    while (n_iter < max_iter) {
      n_iter++;
      if (n_iter == 1) {
        for (int64_t i = 0; i < np; i++) d[i] = -fg[i];
        nold = 0;
        H_diag = 1.f;
      } else {
        // y = g - g_prev, s = d t; y.s > 1e-10 -> history (FIFO of GLUE_HIST)
        float ys = 0.f, yy = 0.f;
        for (int64_t i = 0; i < np; i++) {
          const float yv = fg[i] - pg[i], sv = d[i] * t;
          ys += yv * sv;
          yy += yv * yv;
        }
        if (ys > 1e-10f) {
          if (nold == GLUE_HIST) {  // unreachable with max_iter = 20; kept for the FIFO rule
            for (int h = 0; h + 1 < GLUE_HIST; h++) {
              glue_copy(hs(h), hs(h + 1), np);
              glue_copy(hy(h), hy(h + 1), np);
              ro[h] = ro[h + 1];
            }
            nold--;
          }
          IV hsv = hs(nold), hyv = hy(nold);
          for (int64_t i = 0; i < np; i++) {
            hyv[i] = fg[i] - pg[i];
            hsv[i] = d[i] * t;
          }
          ro[nold] = 1.f / ys;
          nold++;
          H_diag = ys / yy;
        }
        // two-loop recursion
        for (int64_t i = 0; i < np; i++) q[i] = -fg[i];
        for (int h = nold - 1; h >= 0; h--) {
          al[h] = glue_dot(hs(h), q, np) * ro[h];
          IV yv = hy(h);
          for (int64_t i = 0; i < np; i++) q[i] += -al[h] * yv[i];
        }
        for (int64_t i = 0; i < np; i++) d[i] = q[i] * H_diag;
        for (int h = 0; h < nold; h++) {
          const float be = glue_dot(hy(h), d, np) * ro[h];
          IV sv = hs(h);
          for (int64_t i = 0; i < np; i++) d[i] += (al[h] - be) * sv[i];
        }
      }
      glue_copy(pg, fg, np);
      prev_loss = loss;
      if (n_iter == 1) {
        float s1 = 0.f;
        for (int64_t i = 0; i < np; i++) s1 += fabsf(fg[i]);
        t = fminf(1.f, 1.f / s1);
      } else {
        t = 1.f;
      }
      const float gtd = glue_dot(fg, d, np);
      if (gtd > -tol_change) break;
      // ---- _strong_wolfe(obj, x_init, t, d, loss, flat_grad, gtd, max_ls = max_eval - evals)
      glue_copy(xi, x, np);
      const int max_ls = max_eval - evals;
      const float c1 = 1e-4f, c2 = 0.9f;
      float d_norm = 0.f;
      for (int64_t i = 0; i < np; i++) d_norm = fmaxf(d_norm, fabsf(d[i]));
      const double f = loss;
      // buffers: gb[0] = g_new; g_prev starts as flat_grad (fg)
      IV gnew = vec(gb[0]);
      double f_new = eval_at(t, gnew);
      int ls_evals = 1;
      float gtd_new = glue_dot(gnew, d, np);
      float t_prev = 0.f, gtd_prev = gtd;
      double f_prev = f;
      int gprev_buf = -1;  // -1: g_prev is fg
      bool done = false;
      int ls_iter = 0;
      float br[2];
      double bf[2];
      float bgtd[2];
      int bgb[2];  // bracket gradient buffers (-1 = fg)
      int nbr = 0;
      while (ls_iter < max_ls) {
        if ((float)f_new > (float)(f + (double)(c1 * t * gtd)) || (ls_iter > 1 && f_new >= f_prev)) {
          br[0] = t_prev; br[1] = t; bf[0] = f_prev; bf[1] = f_new; bgtd[0] = gtd_prev; bgtd[1] = gtd_new;
          bgb[0] = gprev_buf; bgb[1] = gb[0];
          nbr = 2;
          break;
        }
        if (fabsf(gtd_new) <= -c2 * gtd) {
          br[0] = t; bf[0] = f_new; bgb[0] = gb[0];
          nbr = 1;
          done = true;
          break;
        }
        if (gtd_new >= 0.f) {
          br[0] = t_prev; br[1] = t; bf[0] = f_prev; bf[1] = f_new; bgtd[0] = gtd_prev; bgtd[1] = gtd_new;
          bgb[0] = gprev_buf; bgb[1] = gb[0];
          nbr = 2;
          break;
        }
        const float min_step = t + 0.01f * (t - t_prev), max_step = t * 10.f;
        const float tmp = t;
        t = glue_cubic(t_prev, f_prev, gtd_prev, t, f_new, gtd_new, true, min_step, max_step);
        t_prev = tmp;
        f_prev = f_new;
        // g_prev <- g_new: rotate the buffers so g_new's storage becomes g_prev's
        {
          const int old_prev = gprev_buf;
          gprev_buf = gb[0];
          gb[0] = (old_prev < 0) ? gb[1] : old_prev;
          if (gb[0] == gprev_buf) gb[0] = gb[2];
        }
        gtd_prev = gtd_new;
        gnew = vec(gb[0]);
        f_new = eval_at(t, gnew);
        ls_evals++;
        gtd_new = glue_dot(gnew, d, np);
        ls_iter++;
      }
      if (ls_iter == max_ls) {
        br[0] = 0.f; br[1] = t; bf[0] = f; bf[1] = f_new; bgb[0] = -1; bgb[1] = gb[0];
        bgtd[0] = gtd; bgtd[1] = gtd_new;  // (the reference leaves bracket_gtd unset here)
        nbr = 2;
      }
      int low = 0, high = 1;
      if (nbr == 2) {
        low = bf[0] <= bf[1] ? 0 : 1;
        high = 1 - low;
      }
      bool insuf = false;
      while (!done && ls_iter < max_ls) {
        if (fabsf(br[1] - br[0]) * d_norm < tol_change) break;
        t = glue_cubic(br[0], bf[0], bgtd[0], br[1], bf[1], bgtd[1], false, 0.f, 0.f);
        const float bmax = fmaxf(br[0], br[1]), bmin = fminf(br[0], br[1]);
        const float eps = 0.1f * (bmax - bmin);
        if (fminf(bmax - t, t - bmin) < eps) {
          if (insuf || t >= bmax || t <= bmin) {
            t = (fabsf(t - bmax) < fabsf(t - bmin)) ? bmax - eps : bmin + eps;
            insuf = false;
          } else {
            insuf = true;
          }
        } else {
          insuf = false;
        }
        // a free buffer for g_new: none of the bracket's
        int fb = 6;
        while (fb == bgb[0] || fb == bgb[1]) fb++;
        gnew = vec(fb);
        f_new = eval_at(t, gnew);
        ls_evals++;
        gtd_new = glue_dot(gnew, d, np);
        ls_iter++;
        if ((float)f_new > (float)(f + (double)(c1 * t * gtd)) || f_new >= bf[low]) {
          br[high] = t; bf[high] = f_new; bgb[high] = fb; bgtd[high] = gtd_new;
          low = bf[0] <= bf[1] ? 0 : 1;
          high = 1 - low;
        } else {
          if (fabsf(gtd_new) <= -c2 * gtd) {
            done = true;
          } else if (gtd_new * (br[high] - br[low]) >= 0.f) {
            br[high] = br[low]; bf[high] = bf[low]; bgb[high] = bgb[low]; bgtd[high] = bgtd[low];
          }
          br[low] = t; bf[low] = f_new; bgb[low] = fb; bgtd[low] = gtd_new;
        }
      }
      t = br[low];
      loss = bf[low];
      if (bgb[low] >= 0) glue_copy(fg, vec(bgb[low]), np);  // else flat_grad is already fg
      // ---- back in LBFGS.step
      for (int64_t i = 0; i < np; i++) x[i] = xi[i] + t * d[i];
      amax = 0.f;
      for (int64_t i = 0; i < np; i++) amax = fmaxf(amax, fabsf(fg[i]));
      const bool opt_cond = amax <= tol_grad;
      evals += ls_evals;
      if (n_iter == max_iter) break;
      if (evals >= max_eval) break;
      if (opt_cond) break;
      float dmax = 0.f;
      for (int64_t i = 0; i < np; i++) dmax = fmaxf(dmax, fabsf(d[i] * t));
      if (dmax <= tol_change) break;
      if (fabs(loss - prev_loss) < (double)tol_change) break;
    }
  }
  for (int64_t i = 0; i < np; i++) xout[3 * g0 + i] = glue_wrap(x[i]);
  stats[2 * s] = n_iter;
  stats[2 * s + 1] = evals;
  losses[2 * s] = loss0;
  losses[2 * s + 1] = loss;
}

// ====================================================================== one wave per chain
// k_glue_wave: the same optimiser with the 64 lanes of a wave on one chain.
//
// NeRF as a prefix product.  The frame a placement is made in -- columns bc, nbc, n at the
// last atom c -- turns into the next atom's frame by a rotation that depends on the
// placement offset d alone: bc' = R d^, n' = R normalize(e_x x d^), nbc' = n' x bc'
// (nerf.py:200-207 with ab' = |c - b| bc).  So frame i = frame 2 o A_3 o ... o A_i with
// A_j = (M(d_j), d_j) and (M, o) o (M', o') = (M M', o + M o'): each lane composes a chunk
// of consecutive placements, a wave scan (6 shuffle steps) composes the chunks, each lane
// re-applies its chunk from its prefix.
//
// The gradient without a reverse sweep.  Changing the torsion of atom i rotates atoms
// i, i+1, ... rigidly about the axis bc through c = x_{i-1}; changing its bond angle rotates
// them about -w, w = normalize(bc x (x_i - c)) (the plane b, c, x_i keeps its normal, so the
// next placements follow rigidly).  With the atoms' loss gradients g_m (the frame terms,
// independent per residue):
//   dL/dtorsion_i = bc . (S1_i - c x S0_i),  dL/dangle_i = -w . (S1_i - c x S0_i),
//   S0_i = sum_{m >= i} g_m,  S1_i = sum_{m >= i} x_m x g_m
// -- suffix sums: a chunk sum per lane, a wave suffix scan, a backward walk of the chunk.
//
// The L-BFGS vectors are strided over the lanes (element i on lane i % 64); dot products,
// maxima and the loss are butterfly reductions (the same bits on every lane, so the
// optimiser's control flow stays wave-uniform).  Per-chain scratch sits at the chain's own
// residue / glue offset (memory grows with the residues, not n_chains x the longest chain).
// Parity is statistical, as for k_glue_opt: the exact derivative in float64 instead of
// autograd's float32 chain, other summation orders (tests/test_glue.py bounds).
constexpr int GW = 64;

struct Aff {  // rigid transform: rotation columns c0 c1 c2, offset o
  V3 c0, c1, c2, o;
};
__device__ inline V3 aff_rot(const Aff& A, V3 v) {
  return {A.c0.x * v.x + A.c1.x * v.y + A.c2.x * v.z, A.c0.y * v.x + A.c1.y * v.y + A.c2.y * v.z,
          A.c0.z * v.x + A.c1.z * v.y + A.c2.z * v.z};
}
__device__ inline Aff aff_then(const Aff& A, const Aff& B) {  // A o B
  return {aff_rot(A, B.c0), aff_rot(A, B.c1), aff_rot(A, B.c2), v_addv(A.o, aff_rot(A, B.o))};
}
__device__ inline Aff aff_id() { return {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}}; }
__device__ inline Aff aff_local(V3 d) {  // the placement with offset d in the frame's coordinates
  const V3 e1 = v_scale(d, 1.0 / v_norm(d));
  V3 e3 = {0.0, -e1.z, e1.y};
  e3 = v_scale(e3, 1.0 / v_norm(e3));
  return {e1, v_cross(e3, e1), e3, d};
}
__device__ inline V3 v_shfl(V3 v, int src) { return {__shfl(v.x, src, GW), __shfl(v.y, src, GW), __shfl(v.z, src, GW)}; }
__device__ inline V3 v_shfl_up(V3 v, int k) {
  return {__shfl_up(v.x, k, GW), __shfl_up(v.y, k, GW), __shfl_up(v.z, k, GW)};
}
__device__ inline V3 v_shfl_down(V3 v, int k) {
  return {__shfl_down(v.x, k, GW), __shfl_down(v.y, k, GW), __shfl_down(v.z, k, GW)};
}
__device__ inline Aff aff_shfl_up(const Aff& a, int k) {
  return {v_shfl_up(a.c0, k), v_shfl_up(a.c1, k), v_shfl_up(a.c2, k), v_shfl_up(a.o, k)};
}
__device__ inline double w_sum(double v) {
#pragma unroll
  for (int k = GW / 2; k >= 1; k >>= 1) v += __shfl_xor(v, k, GW);
  return v;
}
__device__ inline float w_sumf(float v) {
#pragma unroll
  for (int k = GW / 2; k >= 1; k >>= 1) v += __shfl_xor(v, k, GW);
  return v;
}
__device__ inline float w_maxf(float v) {
#pragma unroll
  for (int k = GW / 2; k >= 1; k >>= 1) v = fmaxf(v, __shfl_xor(v, k, GW));
  return v;
}

struct WV {  // one float vector of a chain (contiguous at the chain's glue offset)
  float* p;
  __device__ float& operator[](int64_t i) const { return p[i]; }
};

struct GlueWaveProb {
  const int64_t* roff;  // residue offsets [S + 1]
  const double* geo;    // 9 per residue (k_nerf layout)
  const float* tgt;     // 12 per glue
  const int32_t* grid;
  const float* prior;
  const int32_t* kcnt;
  int32_t kmax;
  float lam;
  double wR, wt;
  double* X;    // atoms: 9 per residue, at the residue offset
  double* AX;   // their loss gradients (and the placement offsets during the forward pass)
  float* V;     // GLUE_NVEC vectors of NG (= 3 x glues) floats, each chain at 3 g0
  float* H;     // 2 GLUE_HIST vectors of NG
  int64_t NG;
};

// the (angle, length, torsion) of placement j (atom j + 3) of a chain at parameters x
__device__ inline void glue_wparams(const double* g, WV x, int64_t j, float& A, float& L, float& T) {
  const int64_t k = j / 3;
  const double* gk = g + 9 * k;
  const double* gn = gk + 9;
  const int m = (int)(j - 3 * k);
  if (m == 0) {
    A = (float)gk[4], L = (float)gk[3], T = (float)gk[6];
  } else if (m == 1) {
    A = glue_wrap(x[3 * k + 1]), L = (float)gn[0], T = glue_wrap(x[3 * k]);
  } else {
    A = (float)gn[2], L = (float)gn[1], T = glue_wrap(x[3 * k + 2]);
  }
}

// loss and gradient of one chain (r >= 2 residues) at x, by the wave; grad written in full
// (one out-of-line copy: the optimiser calls it from four places)
__device__ __attribute__((noinline)) double glue_eval_wave(const GlueWaveProb& P, int64_t a0, int64_t r, const double* g, const float* tg,
                                 const float* pr, const int32_t* kc, WV x, WV grad) {
  const int lane = threadIdx.x;
  double* X = P.X + 9 * a0;
  double* AX = P.AX + 9 * a0;
  const int64_t n = 3 * (r - 1);  // placements (atoms 3 .. 3r - 1)
  const int64_t CH = (n + GW - 1) / GW;
  const int64_t j0 = min(n, (int64_t)lane * CH), j1 = min(n, j0 + CH);
  __syncthreads();  // (x was written lane-strided)
  // -- forward: this lane's chunk of placements, composed; offsets kept in AX meanwhile
  Aff T = aff_id();
  for (int64_t j = j0; j < j1; j++) {
    float A, L, Tq;
    glue_wparams(g, x, j, A, L, Tq);
    float f0, f1, f2;
    glue_d(A, L, Tq, f0, f1, f2);
    const V3 d = {(double)f0, (double)f1, (double)f2};
    stx(AX, 1, j + 3, d);
    T = aff_then(T, aff_local(d));
  }
#pragma unroll
  for (int k = 1; k < GW; k <<= 1) {
    const Aff u = aff_shfl_up(T, k);
    if (lane >= k) T = aff_then(u, T);
  }
  Aff F = aff_shfl_up(T, 1);  // exclusive prefix
  if (lane == 0) F = aff_id();
  V3 p3, p2, p1;
  backbone_start(g[1], g[0], g[2], p3, p2, p1);
  if (lane == 0) {
    stx(X, 1, 0, p3);
    stx(X, 1, 1, p2);
    stx(X, 1, 2, p1);
  }
  {
    const V3 bc = v_scale(v_sub(p1, p2), 1.0 / v_norm(v_sub(p1, p2)));
    const V3 m = v_cross(v_sub(p2, p3), bc);
    const V3 nn = v_scale(m, 1.0 / v_norm(m));
    const Aff F2 = {bc, v_cross(nn, bc), nn, p1};
    F = aff_then(F2, F);
  }
  for (int64_t j = j0; j < j1; j++) {
    F = aff_then(F, aff_local(ldx(AX, 1, j + 3)));
    stx(X, 1, j + 3, F.o);
  }
  __syncthreads();
  // -- frames of residues 1..r-1 against the targets (bpe.py:539-548), lane-strided
  double rot = 0.0, trans = 0.0;
  for (int64_t i = 1 + lane; i < r; i += GW) {
    const V3 N = ldx(X, 1, 3 * i), CA = ldx(X, 1, 3 * i + 1), C = ldx(X, 1, 3 * i + 2);
    const float* Tg = tg + 12 * (i - 1);
    const V3 vx = v_sub(C, CA), vu = v_sub(N, CA);
    const V3 ex = glue_normalize(vx), eu = glue_normalize(vu);
    const V3 w = v_cross(ex, eu);
    const V3 ez = glue_normalize(w);
    const V3 ey = v_cross(ez, ex);
    const V3 Rx = {Tg[0], Tg[3], Tg[6]}, Ry = {Tg[1], Tg[4], Tg[7]}, Rz = {Tg[2], Tg[5], Tg[8]},
             Rt = {Tg[9], Tg[10], Tg[11]};
    const V3 dx = v_sub(ex, Rx), dy = v_sub(ey, Ry), dz = v_sub(ez, Rz), dt = v_sub(CA, Rt);
    rot += 0.5 * (v_dot(dx, dx) + v_dot(dy, dy) + v_dot(dz, dz));
    trans += v_dot(dt, dt);
    V3 gx = v_scale(dx, P.wR), gy = v_scale(dy, P.wR), gz = v_scale(dz, P.wR);
    gz = v_addv(gz, v_cross(ex, gy));
    gx = v_addv(gx, v_cross(gy, ez));
    const V3 gw = glue_normalize_back(w, gz);
    gx = v_addv(gx, v_cross(eu, gw));
    const V3 gu = v_cross(gw, ex);
    const V3 gvx = glue_normalize_back(vx, gx), gvu = glue_normalize_back(vu, gu);
    stx(AX, 1, 3 * i + 2, gvx);
    stx(AX, 1, 3 * i, gvu);
    stx(AX, 1, 3 * i + 1, v_addv(v_scale(v_addv(gvx, gvu), -1.0), v_scale(dt, 2.0 * P.wt)));
  }
  // -- prior (bpe.py:527-534, 549-558), float32, glue-strided: the gradient starts from it
  float prior = 0.f;
  for (int64_t k = lane; k + 1 < r; k += GW) {
    float term = 0.f;
    for (int t = 0; t < 3; t++) {
      float gp = 0.f;
      if (P.lam != 0.f) {
        const float a = glue_wrap(x[3 * k + t]);
        const float kappa = t == 0 ? 50.f : 20.f;
        const float* cen = pr + (2 * t) * P.kmax;
        const float* wt = cen + P.kmax;
        float mx = -INFINITY;
        for (int jj = 0; jj < kc[t]; jj++) mx = fmaxf(mx, kappa * f_cos(a - cen[jj]) + f_log(wt[jj] + 1e-12f));
        float se = 0.f, sg = 0.f;
        for (int jj = 0; jj < kc[t]; jj++) {
          const float e = f_exp(kappa * f_cos(a - cen[jj]) + f_log(wt[jj] + 1e-12f) - mx);
          se += e;
          sg += e * kappa * f_sin(a - cen[jj]);
        }
        term += -(mx + f_log(se));
        gp = P.lam * (sg / se);
      }
      grad[3 * k + t] = gp;
    }
    prior += term;
  }
  __syncthreads();
  // -- the parameters' gradients from suffix sums of g_m and x_m x g_m over the atoms
  V3 S0 = {0, 0, 0}, S1 = {0, 0, 0};
  for (int64_t j = j0; j < j1; j++) {
    const V3 gm = ldx(AX, 1, j + 3), xm = ldx(X, 1, j + 3);
    S0 = v_addv(S0, gm);
    S1 = v_addv(S1, v_cross(xm, gm));
  }
#pragma unroll
  for (int k = 1; k < GW; k <<= 1) {
    const V3 u0 = v_shfl_down(S0, k), u1 = v_shfl_down(S1, k);
    if (lane + k < GW) {
      S0 = v_addv(S0, u0);
      S1 = v_addv(S1, u1);
    }
  }
  {  // exclusive: the lanes after this one
    const V3 u0 = v_shfl_down(S0, 1), u1 = v_shfl_down(S1, 1);
    S0 = lane + 1 < GW ? u0 : V3{0, 0, 0};
    S1 = lane + 1 < GW ? u1 : V3{0, 0, 0};
  }
  if (j1 > j0) {
    V3 xi = ldx(X, 1, j1 - 1 + 3), c = ldx(X, 1, j1 - 1 + 2), b = ldx(X, 1, j1 - 1 + 1);
    for (int64_t j = j1 - 1; j >= j0; j--) {
      const V3 gm = ldx(AX, 1, j + 3);
      S0 = v_addv(S0, gm);
      S1 = v_addv(S1, v_cross(xi, gm));
      const int64_t k = j / 3;
      const int m = (int)(j - 3 * k);
      if (m != 0) {
        const V3 u = v_sub(c, b);
        const V3 bc = v_scale(u, 1.0 / v_norm(u));
        const V3 v = v_sub(S1, v_cross(c, S0));
        const float gT = (float)v_dot(bc, v);
        if (m == 1) {  // CA_{k+1}: torsion omega_k, angle C:1N:1CA_k
          const V3 wv = v_cross(bc, v_sub(xi, c));
          const float gA = (float)(-v_dot(v_scale(wv, 1.0 / v_norm(wv)), v));
          grad[3 * k] = glue_wrap_back(x[3 * k], grad[3 * k] + gT);
          grad[3 * k + 1] = glue_wrap_back(x[3 * k + 1], grad[3 * k + 1] + gA);
        } else {  // C_{k+1}: torsion phi_{k+1}
          grad[3 * k + 2] = glue_wrap_back(x[3 * k + 2], grad[3 * k + 2] + gT);
        }
      }
      if (j > j0) {  // one atom back
        xi = c;
        c = b;
        b = ldx(X, 1, j);
      }
    }
  }
  double loss = P.wR * w_sum(rot) + P.wt * w_sum(trans);
  const float pri = w_sumf(prior);
  if (P.lam != 0.f) loss += (double)(P.lam * pri);
  __syncthreads();
  return loss;
}

__device__ inline float w_dot(WV a, WV b, int64_t n) {
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += GW) s += a[i] * b[i];
  return w_sumf(s);
}
__device__ inline void w_copy(WV dst, WV src, int64_t n) {
  for (int64_t i = threadIdx.x; i < n; i += GW) dst[i] = src[i];
}

// one chain per 64-thread workgroup; the control flow of k_glue_opt (torch/optim/lbfgs.py),
// every scalar wave-uniform
__global__ __launch_bounds__(GW) void k_glue_wave(GlueWaveProb P, int64_t S, const float* x0, float* xout,
                                                  int32_t* stats, double* losses) {
  const int64_t s = blockIdx.x;
  const int lane = threadIdx.x;
  if (s >= S) return;
  const int64_t a0 = P.roff[s], r = P.roff[s + 1] - a0;
  const int64_t np = 3 * (r - 1), g0 = a0 - s;
  if (r < 2) {
    if (lane == 0) {
      stats[2 * s] = 0;
      stats[2 * s + 1] = 0;
      losses[2 * s] = 0.0;
      losses[2 * s + 1] = 0.0;
    }
    return;
  }
  const double* g = P.geo + 9 * a0;
  const float* tg = P.tgt + 12 * g0;
  const int32_t gi = P.grid[s];
  const float* pr = P.prior + (int64_t)gi * 6 * P.kmax;
  const int32_t* kc = P.kcnt + 3 * gi;
  auto vec = [&](int v) { return WV{P.V + (int64_t)v * P.NG + 3 * g0}; };
  auto hs = [&](int h) { return WV{P.H + (int64_t)h * P.NG + 3 * g0}; };
  auto hy = [&](int h) { return WV{P.H + (int64_t)(GLUE_HIST + h) * P.NG + 3 * g0}; };
  WV x = vec(0), d = vec(1), fg = vec(2), pg = vec(3), xi = vec(4), q = vec(5);
  int gb[3] = {6, 7, 8};
  __shared__ float ro[GLUE_HIST], al[GLUE_HIST];  // (wave-uniform values: every lane writes the same)
  int nold = 0;
  for (int64_t i = lane; i < np; i += GW) x[i] = x0[3 * g0 + i];
  auto eval_at = [&](float t, WV out) -> double {
    for (int64_t i = lane; i < np; i += GW) q[i] = xi[i] + t * d[i];
    return glue_eval_wave(P, a0, r, g, tg, pr, kc, q, out);
  };
  auto vmaxabs = [&](WV v) {
    float m = 0.f;
    for (int64_t i = lane; i < np; i += GW) m = fmaxf(m, fabsf(v[i]));
    return w_maxf(m);
  };
  double loss = glue_eval_wave(P, a0, r, g, tg, pr, kc, x, fg);
  const double loss0 = loss;
  int evals = 1, n_iter = 0;
  float amax = vmaxabs(fg);
  const float tol_grad = 1e-7f, tol_change = 1e-9f;
  const int max_iter = 20, max_eval = 25;
  float t = 1.f, H_diag = 1.f;
  double prev_loss = loss;
  if (!(amax <= tol_grad)) {
    while (n_iter < max_iter) {
      n_iter++;
      if (n_iter == 1) {
        for (int64_t i = lane; i < np; i += GW) d[i] = -fg[i];
        nold = 0;
        H_diag = 1.f;
      } else {
        float ys = 0.f, yy = 0.f;
        for (int64_t i = lane; i < np; i += GW) {
          const float yv = fg[i] - pg[i], sv = d[i] * t;
          ys += yv * sv;
          yy += yv * yv;
        }
        ys = w_sumf(ys);
        yy = w_sumf(yy);
        if (ys > 1e-10f) {
          if (nold == GLUE_HIST) {  // unreachable with max_iter = 20; kept for the FIFO rule
            for (int h = 0; h + 1 < GLUE_HIST; h++) {
              w_copy(hs(h), hs(h + 1), np);
              w_copy(hy(h), hy(h + 1), np);
              ro[h] = ro[h + 1];
            }
            nold--;
          }
          const WV hsv = hs(nold), hyv = hy(nold);
          for (int64_t i = lane; i < np; i += GW) {
            hyv[i] = fg[i] - pg[i];
            hsv[i] = d[i] * t;
          }
          ro[nold] = 1.f / ys;
          nold++;
          H_diag = ys / yy;
        }
        for (int64_t i = lane; i < np; i += GW) q[i] = -fg[i];
        for (int h = nold - 1; h >= 0; h--) {
          al[h] = w_dot(hs(h), q, np) * ro[h];
          const WV yv = hy(h);
          for (int64_t i = lane; i < np; i += GW) q[i] += -al[h] * yv[i];
        }
        for (int64_t i = lane; i < np; i += GW) d[i] = q[i] * H_diag;
        for (int h = 0; h < nold; h++) {
          const float be = w_dot(hy(h), d, np) * ro[h];
          const WV sv = hs(h);
          for (int64_t i = lane; i < np; i += GW) d[i] += (al[h] - be) * sv[i];
        }
      }
      w_copy(pg, fg, np);
      prev_loss = loss;
      if (n_iter == 1) {
        float s1 = 0.f;
        for (int64_t i = lane; i < np; i += GW) s1 += fabsf(fg[i]);
        t = fminf(1.f, 1.f / w_sumf(s1));
      } else {
        t = 1.f;
      }
      const float gtd = w_dot(fg, d, np);
      if (gtd > -tol_change) break;
      // ---- _strong_wolfe
      w_copy(xi, x, np);
      const int max_ls = max_eval - evals;
      const float c1 = 1e-4f, c2 = 0.9f;
      const float d_norm = vmaxabs(d);
      const double f = loss;
      WV gnew = vec(gb[0]);
      double f_new = eval_at(t, gnew);
      int ls_evals = 1;
      float gtd_new = w_dot(gnew, d, np);
      float t_prev = 0.f, gtd_prev = gtd;
      double f_prev = f;
      int gprev_buf = -1;
      bool done = false;
      int ls_iter = 0;
      float br[2];
      double bf[2];
      float bgtd[2];
      int bgb[2];
      int nbr = 0;
      while (ls_iter < max_ls) {
        if ((float)f_new > (float)(f + (double)(c1 * t * gtd)) || (ls_iter > 1 && f_new >= f_prev)) {
          br[0] = t_prev; br[1] = t; bf[0] = f_prev; bf[1] = f_new; bgtd[0] = gtd_prev; bgtd[1] = gtd_new;
          bgb[0] = gprev_buf; bgb[1] = gb[0];
          nbr = 2;
          break;
        }
        if (fabsf(gtd_new) <= -c2 * gtd) {
          br[0] = t; bf[0] = f_new; bgb[0] = gb[0];
          nbr = 1;
          done = true;
          break;
        }
        if (gtd_new >= 0.f) {
          br[0] = t_prev; br[1] = t; bf[0] = f_prev; bf[1] = f_new; bgtd[0] = gtd_prev; bgtd[1] = gtd_new;
          bgb[0] = gprev_buf; bgb[1] = gb[0];
          nbr = 2;
          break;
        }
        const float min_step = t + 0.01f * (t - t_prev), max_step = t * 10.f;
        const float tmp = t;
        t = glue_cubic(t_prev, f_prev, gtd_prev, t, f_new, gtd_new, true, min_step, max_step);
        t_prev = tmp;
        f_prev = f_new;
        {
          const int old_prev = gprev_buf;
          gprev_buf = gb[0];
          gb[0] = (old_prev < 0) ? gb[1] : old_prev;
          if (gb[0] == gprev_buf) gb[0] = gb[2];
        }
        gtd_prev = gtd_new;
        gnew = vec(gb[0]);
        f_new = eval_at(t, gnew);
        ls_evals++;
        gtd_new = w_dot(gnew, d, np);
        ls_iter++;
      }
      if (ls_iter == max_ls) {
        br[0] = 0.f; br[1] = t; bf[0] = f; bf[1] = f_new; bgb[0] = -1; bgb[1] = gb[0];
        bgtd[0] = gtd; bgtd[1] = gtd_new;
        nbr = 2;
      }
      int low = 0, high = 1;
      if (nbr == 2) {
        low = bf[0] <= bf[1] ? 0 : 1;
        high = 1 - low;
      }
      bool insuf = false;
      while (!done && ls_iter < max_ls) {
        if (fabsf(br[1] - br[0]) * d_norm < tol_change) break;
        t = glue_cubic(br[0], bf[0], bgtd[0], br[1], bf[1], bgtd[1], false, 0.f, 0.f);
        const float bmax = fmaxf(br[0], br[1]), bmin = fminf(br[0], br[1]);
        const float eps = 0.1f * (bmax - bmin);
        if (fminf(bmax - t, t - bmin) < eps) {
          if (insuf || t >= bmax || t <= bmin) {
            t = (fabsf(t - bmax) < fabsf(t - bmin)) ? bmax - eps : bmin + eps;
            insuf = false;
          } else {
            insuf = true;
          }
        } else {
          insuf = false;
        }
        int fb = 6;
        while (fb == bgb[0] || fb == bgb[1]) fb++;
        gnew = vec(fb);
        f_new = eval_at(t, gnew);
        ls_evals++;
        gtd_new = w_dot(gnew, d, np);
        ls_iter++;
        if ((float)f_new > (float)(f + (double)(c1 * t * gtd)) || f_new >= bf[low]) {
          br[high] = t; bf[high] = f_new; bgb[high] = fb; bgtd[high] = gtd_new;
          low = bf[0] <= bf[1] ? 0 : 1;
          high = 1 - low;
        } else {
          if (fabsf(gtd_new) <= -c2 * gtd) {
            done = true;
          } else if (gtd_new * (br[high] - br[low]) >= 0.f) {
            br[high] = br[low]; bf[high] = bf[low]; bgb[high] = bgb[low]; bgtd[high] = bgtd[low];
          }
          br[low] = t; bf[low] = f_new; bgb[low] = fb; bgtd[low] = gtd_new;
        }
      }
      t = br[low];
      loss = bf[low];
      if (bgb[low] >= 0) w_copy(fg, vec(bgb[low]), np);
      for (int64_t i = lane; i < np; i += GW) x[i] = xi[i] + t * d[i];
      amax = vmaxabs(fg);
      const bool opt_cond = amax <= tol_grad;
      evals += ls_evals;
      if (n_iter == max_iter) break;
      if (evals >= max_eval) break;
      if (opt_cond) break;
      float dmax = 0.f;
      for (int64_t i = lane; i < np; i += GW) dmax = fmaxf(dmax, fabsf(d[i] * t));
      if (w_maxf(dmax) <= tol_change) break;
      if (fabs(loss - prev_loss) < (double)tol_change) break;
    }
  }
  for (int64_t i = lane; i < np; i += GW) xout[3 * g0 + i] = glue_wrap(x[i]);
  if (lane == 0) {
    stats[2 * s] = n_iter;
    stats[2 * s + 1] = evals;
    losses[2 * s] = loss0;
    losses[2 * s + 1] = loss;
  }
}

}  // namespace gb
