// rmsd.h -- Kabsch RMSD of structure pairs (the RMSD
// partitioning's k-medoids distance matrix, foldingdiff/algo.py:144-213, and the
// per-occurrence medoid assignment, bpe.py:645-657,1764-1777).  Included once by
// geobpe.hip.
//
// compute_rmsd(P, Q) (algo.py:48-65) aligns Q onto P with kabsch (algo.py:8-46):
// H = Pc^T Qc, SVD H = U S Vt, R = U Vt with the last row of Vt negated when
// det(R) < 0, Q_aligned = Qc R^T + centroid(P), RMSD = sqrt(mean |P - Q_aligned|^2).
// Here, float64, one thread per pair: centroids and centred coordinates are
// computed once per structure; per pair the 3x3 H, a cyclic Jacobi
// eigen-decomposition of H^T H = V diag(s^2) V^T, U's columns H v_i / s_i (the
// third as u1 x u2, so det U = +1; v3 sign-fixed so det V = +1: the reflection
// correction), R = U V^T, then the explicit residual sum |pc - R qc|^2 -- the
// reference's own arithmetic path (no E0 - 2 sum(s) cancellation), so tiny RMSDs
// agree to ~1e-15 absolute.  Degenerate H (collinear or coincident atoms) takes
// an arbitrary orthonormal completion: the RMSD is the same for every optimal R.
#pragma once

namespace gb {

__device__ inline void jacobi3(double A[3][3], double V[3][3]) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) V[i][j] = i == j ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 24; sweep++) {
    const double off = A[0][1] * A[0][1] + A[0][2] * A[0][2] + A[1][2] * A[1][2];
    const double dia = A[0][0] * A[0][0] + A[1][1] * A[1][1] + A[2][2] * A[2][2];
    if (off <= 1e-36 * dia || off == 0.0) break;
    for (int p = 0; p < 2; p++)
      for (int q = p + 1; q < 3; q++) {
        const double apq = A[p][q];
        if (apq == 0.0) continue;
        const double theta = (A[q][q] - A[p][p]) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 3; k++) {  // A <- J^T A J
          const double akp = A[k][p], akq = A[k][q];
          A[k][p] = c * akp - s * akq;
          A[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < 3; k++) {
          const double apk = A[p][k], aqk = A[q][k];
          A[p][k] = c * apk - s * aqk;
          A[q][k] = s * apk + c * aqk;
        }
        for (int k = 0; k < 3; k++) {
          const double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = c * vkp - s * vkq;
          V[k][q] = s * vkp + c * vkq;
        }
      }
  }
}

__device__ inline void unit_perp(const double u[3], double out[3]) {  // any unit vector orthogonal to u
  const int m = fabs(u[0]) <= fabs(u[1]) && fabs(u[0]) <= fabs(u[2]) ? 0 : (fabs(u[1]) <= fabs(u[2]) ? 1 : 2);
  double e[3] = {0, 0, 0};
  e[m] = 1.0;
  double w[3] = {u[1] * e[2] - u[2] * e[1], u[2] * e[0] - u[0] * e[2], u[0] * e[1] - u[1] * e[0]};
  const double n = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  for (int k = 0; k < 3; k++) out[k] = w[k] / n;
}

// the optimal proper rotation R (q -> p) of the covariance H = sum p q^T
__device__ inline void kabsch_rotation(const double H[3][3], double R[3][3]) {
  double A[3][3], V[3][3];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) A[i][j] = H[0][i] * H[0][j] + H[1][i] * H[1][j] + H[2][i] * H[2][j];  // H^T H
  jacobi3(A, V);
  // eigenvalues descending (selection on 3 values), columns of V along
  int o[3] = {0, 1, 2};
  for (int i = 0; i < 2; i++)
    for (int j = i + 1; j < 3; j++)
      if (A[o[j]][o[j]] > A[o[i]][o[i]]) {
        const int t = o[i];
        o[i] = o[j];
        o[j] = t;
      }
  double v[3][3], u[3][3];  // v[i] = i-th right singular vector
  for (int i = 0; i < 3; i++)
    for (int k = 0; k < 3; k++) v[i][k] = V[k][o[i]];
  const double s1 = sqrt(fmax(A[o[0]][o[0]], 0.0));
  for (int i = 0; i < 2; i++) {
    double hv[3];
    for (int k = 0; k < 3; k++) hv[k] = H[k][0] * v[i][0] + H[k][1] * v[i][1] + H[k][2] * v[i][2];
    const double n = sqrt(hv[0] * hv[0] + hv[1] * hv[1] + hv[2] * hv[2]);
    if (n > 1e-12 * fmax(s1, 1e-300)) {
      for (int k = 0; k < 3; k++) u[i][k] = hv[k] / n;
      if (i == 1) {  // re-orthogonalise against u1
        const double d = u[1][0] * u[0][0] + u[1][1] * u[0][1] + u[1][2] * u[0][2];
        for (int k = 0; k < 3; k++) u[1][k] -= d * u[0][k];
        const double m = sqrt(u[1][0] * u[1][0] + u[1][1] * u[1][1] + u[1][2] * u[1][2]);
        if (m > 1e-12)
          for (int k = 0; k < 3; k++) u[1][k] /= m;
        else
          unit_perp(u[0], u[1]);
      }
    } else if (i == 0) {  // H ~ 0: any rotation
      u[0][0] = 1;
      u[0][1] = 0;
      u[0][2] = 0;
    } else {
      unit_perp(u[0], u[1]);
    }
  }
  u[2][0] = u[0][1] * u[1][2] - u[0][2] * u[1][1];
  u[2][1] = u[0][2] * u[1][0] - u[0][0] * u[1][2];
  u[2][2] = u[0][0] * u[1][1] - u[0][1] * u[1][0];
  // det V = +1 (v3 = v1 x v2): R = sum u_i v_i^T is then a proper rotation
  v[2][0] = v[0][1] * v[1][2] - v[0][2] * v[1][1];
  v[2][1] = v[0][2] * v[1][0] - v[0][0] * v[1][2];
  v[2][2] = v[0][0] * v[1][1] - v[0][1] * v[1][0];
  for (int a = 0; a < 3; a++)
    for (int b = 0; b < 3; b++) R[a][b] = u[0][a] * v[0][b] + u[1][a] * v[1][b] + u[2][a] * v[2][b];
}

// centred coordinates (n structures x L atoms x 3) in place; one thread per structure
__global__ __launch_bounds__(BLOCK) void k_rmsd_center(double* xyz, int32_t n, int32_t L) {
  const int32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  double* p = xyz + (int64_t)s * L * 3;
  double c[3] = {0, 0, 0};
  for (int32_t i = 0; i < L; i++)
    for (int k = 0; k < 3; k++) c[k] += p[3 * i + k];
  for (int k = 0; k < 3; k++) c[k] /= L;
  for (int32_t i = 0; i < L; i++)
    for (int k = 0; k < 3; k++) p[3 * i + k] -= c[k];
}

// out[i * nb + j] = RMSD(A_i, B_j) (P = A_i, Q = B_j); symmetric: A == B and only
// j >= i is computed and mirrored (the reference's upper-triangle loop)
__global__ __launch_bounds__(BLOCK) void k_rmsd_pairs(const double* A, const double* B, int32_t na, int32_t nb,
                                                      int32_t L, int symmetric, double* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)na * nb) return;
  const int32_t i = (int32_t)(t / nb), j = (int32_t)(t % nb);
  if (symmetric && j < i) return;
  const double* p = A + (int64_t)i * L * 3;
  const double* q = B + (int64_t)j * L * 3;
  double H[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
  for (int32_t a = 0; a < L; a++) {
    const double px = p[3 * a], py = p[3 * a + 1], pz = p[3 * a + 2];
    const double qx = q[3 * a], qy = q[3 * a + 1], qz = q[3 * a + 2];
    H[0][0] += px * qx;
    H[0][1] += px * qy;
    H[0][2] += px * qz;
    H[1][0] += py * qx;
    H[1][1] += py * qy;
    H[1][2] += py * qz;
    H[2][0] += pz * qx;
    H[2][1] += pz * qy;
    H[2][2] += pz * qz;
  }
  double R[3][3];
  kabsch_rotation(H, R);
  double ss = 0;
  for (int32_t a = 0; a < L; a++) {
    const double qx = q[3 * a], qy = q[3 * a + 1], qz = q[3 * a + 2];
    for (int k = 0; k < 3; k++) {
      const double d = p[3 * a + k] - (R[k][0] * qx + R[k][1] * qy + R[k][2] * qz);
      ss += d * d;
    }
  }
  const double r = sqrt(ss / L);
  out[t] = r;
  if (symmetric && j != i) out[(int64_t)j * nb + i] = r;
}

}  // namespace gb

namespace gb {

// ------------------------------------------------------------------ NeRF
// Token coordinates from internal coordinates (Tokenizer.compute_coords ->
// Tokenizer.geo_nerf, tokenizer.py:317-363; NERFBuilder.cartesian_coords and
// place_dihedral, nerf.py:85-211; the first residue by update_backbone_positions,
// angles_and_coords.py:238-316).  One thread per span (a span = whole residues,
// 3r - 1 bonds).  geo: 9 float64 per residue k of a span,
//   {N:CA_k, CA:C_k, tau_k, 0C:1N_k, CA:C:1N_k, C:1N:1CA_k, psi_k, omega_k, phi_k}
// (the last six are the junction to residue k + 1, unused for the span's last
// residue); out: N, CA, C of every residue (9 float64).
__device__ inline V3 v_unit(V3 a) { return v_scale(a, 1.0 / v_norm(a)); }
__device__ inline V3 v_add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }

__device__ inline V3 place_dihedral(V3 a, V3 b, V3 c, double angle, double len, double torsion) {
  const V3 ab = v_sub(b, a);
  const V3 bc = v_unit(v_sub(c, b));
  const V3 n = v_unit(v_cross(ab, bc));
  const V3 nbc = v_cross(n, bc);
  const double d0 = -len * cos(angle), d1 = len * cos(torsion) * sin(angle), d2 = len * sin(torsion) * sin(angle);
  // m = [bc | nbc | n] (columns), m . d + c
  return {bc.x * d0 + nbc.x * d1 + n.x * d2 + c.x, bc.y * d0 + nbc.y * d1 + n.y * d2 + c.y,
          bc.z * d0 + nbc.z * d1 + n.z * d2 + c.z};
}

// Rodrigues: v cos + (k x v) sin + k (k . v)(1 - cos)
__device__ inline V3 rotate_vec(V3 v, V3 k, double ang) {
  const double c = cos(ang), s = sin(ang);
  const V3 kv = v_cross(k, v);
  const double kd = v_dot(k, v) * (1.0 - c);
  return {v.x * c + kv.x * s + k.x * kd, v.y * c + kv.y * s + k.y * kd, v.z * c + kv.z * s + k.z * kd};
}

// the first residue: C fixed, CA on the C->CA line at L_CA_C, N rotated in the
// N-CA-C plane to the angle theta and rescaled to L_N_CA
__device__ inline void backbone_start(double l_ca_c, double l_n_ca, double theta, V3& N, V3& CA, V3& C) {
  const V3 n0 = {17.047, 14.099, 3.625}, ca0 = {16.967, 12.784, 4.338}, c0 = {15.685, 12.755, 5.133};  // nerf.py N/CA/C_INIT (1CRN)
  const V3 v = v_unit(v_sub(ca0, c0));
  CA = v_add(c0, v_scale(v, l_ca_c));
  const V3 vn = v_sub(n0, CA), vc = v_sub(c0, CA);
  double ct = v_dot(vn, vc) / (v_norm(vn) * v_norm(vc));
  ct = fmin(fmax(ct, -1.0), 1.0);
  const double dtheta = theta - acos(ct);
  const V3 axis = v_unit(v_cross(vn, vc));
  V3 r = rotate_vec(vn, axis, -dtheta);
  r = v_scale(r, l_n_ca / v_norm(r));
  N = v_add(CA, r);
  C = c0;
}

__global__ __launch_bounds__(BLOCK) void k_nerf(int64_t n_spans, const int64_t* res_off, const double* geo,
                                                double* out) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_spans) return;
  const int64_t a = res_off[s], r = res_off[s + 1] - a;
  if (r <= 0) return;
  const double* g = geo + 9 * a;
  double* o = out + 9 * a;
  V3 p3, p2, p1;  // the last three atoms placed: ..., p3, p2, p1
  backbone_start(g[1], g[0], g[2], p3, p2, p1);
  auto put = [&](int64_t atom, V3 v) {
    o[3 * atom] = v.x;
    o[3 * atom + 1] = v.y;
    o[3 * atom + 2] = v.z;
  };
  put(0, p3);
  put(1, p2);
  put(2, p1);
  for (int64_t k = 0; k + 1 < r; k++) {
    const double* gk = g + 9 * k;
    const double* gn = g + 9 * (k + 1);
    // (C, N): CA:C:1N_k, 0C:1N_k, psi_k; (N, CA): C:1N:1CA_k, N:CA_{k+1}, omega_k;
    // (CA, C): tau_{k+1}, CA:C_{k+1}, phi_k
    const V3 nN = place_dihedral(p3, p2, p1, gk[4], gk[3], gk[6]);
    const V3 nCA = place_dihedral(p2, p1, nN, gk[5], gn[0], gk[7]);
    const V3 nC = place_dihedral(p1, nN, nCA, gn[2], gn[1], gk[8]);
    put(3 * (k + 1), nN);
    put(3 * (k + 1) + 1, nCA);
    put(3 * (k + 1) + 2, nC);
    p3 = nN;
    p2 = nCA;
    p1 = nC;
  }
}

}  // namespace gb
