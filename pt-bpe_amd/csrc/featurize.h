// featurize.h -- PDB backbone -> the reference's internal-coordinate frame
// (SURVEY.md §8(f) row 2).  Included once by geobpe.hip.
//
// Host: a fixed-column PDB reader for the backbone (N, CA, C of every amino-acid
// residue of the first model; the first alternate location of an atom) --
// PDBFile.read + get_structure(model=1) + filter_backbone of the reference's
// canonical_distances_and_dihedrals (angles_and_coords.py:69-154, biotite).
// Device: one thread per residue computes the nine columns with the reference's
// index conventions (angles_and_coords.py:100-154):
//   row r of a chain of n residues (N_r, CA_r, C_r):
//   phi[r]      = dihedral(C_{r-1}, N_r, CA_r, C_r)        r >= 1   (NaN at 0)
//   psi[r]      = dihedral(N_r, CA_r, C_r, N_{r+1})        r <= n-2 (NaN last)
//   omega[r]    = dihedral(CA_r, C_r, N_{r+1}, CA_{r+1})   r <= n-2 (NaN last)
//   tau[r]      = angle(N_{r+1}, CA_{r+1}, C_{r+1})        r <= n-2 (NaN last: the 0-index pad)
//   CA:C:1N[r]  = angle(CA_r, C_r, N_{r+1})                r <= n-2 (NaN last)
//   C:1N:1CA[r] = angle(C_r, N_{r+1}, CA_{r+1})            r <= n-2 (NaN last)
//   0C:1N[r]    = |N_{r+1} - C_r|                          r <= n-2 (0 last)
//   N:CA[r]     = |CA_{r+1} - N_{r+1}|                     r <= n-2 (0 last)
//   CA:C[r]     = |C_{r+1} - CA_{r+1}|                     r <= n-2 (0 last)
// dihedral / angle follow biotite.structure.geometry (unit bond vectors, atan2 of
// the normal frame; arccos of the normalised dot product).  Parity against
// biotite itself is UNPINNED here (biotite is not installed): the tests check the
// kernel against a float64 numpy restatement and NeRF round trips.
#pragma once

#include <cctype>
#include <fstream>
#include <set>
#include <sstream>
#include <string>
#include <vector>

namespace gb {

struct V3 {
  double x, y, z;
};
__device__ inline V3 v_sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ inline double v_dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ inline V3 v_cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
__device__ inline double v_norm(V3 a) { return sqrt(v_dot(a, a)); }
__device__ inline V3 v_scale(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }

// biotite.structure.dihedral
__device__ inline double bb_dihedral(V3 p1, V3 p2, V3 p3, V3 p4) {
  V3 b1 = v_sub(p2, p1), b2 = v_sub(p3, p2), b3 = v_sub(p4, p3);
  b1 = v_scale(b1, 1.0 / v_norm(b1));
  b2 = v_scale(b2, 1.0 / v_norm(b2));
  b3 = v_scale(b3, 1.0 / v_norm(b3));
  const V3 n1 = v_cross(b1, b2), n2 = v_cross(b2, b3);
  const double x = v_dot(n1, n2);
  const double y = v_dot(v_cross(n1, n2), b2);
  return atan2(y, x);
}
// biotite.structure.angle: at the middle atom
__device__ inline double bb_angle(V3 a, V3 b, V3 c) {
  const V3 v1 = v_sub(a, b), v2 = v_sub(c, b);
  return acos(v_dot(v1, v2) / (v_norm(v1) * v_norm(v2)));
}

// xyz: per residue N, CA, C (9 doubles); cols: the nine columns in
// include/geobpe.h GEOBPE_COL_* order
__global__ __launch_bounds__(BLOCK) void k_featurize(int64_t nrows, const int64_t* row_off, const double* xyz,
                                                     double* out, int64_t R) {
  for (int64_t row = blockIdx.x; row < nrows; row += gridDim.x) {
    const int64_t a = row_off[row], b = row_off[row + 1];
    const int64_t n = b - a;
    for (int64_t r = threadIdx.x; r < n; r += blockDim.x) {
      auto at = [&](int64_t res, int k) {
        const double* p = xyz + 9 * (a + res) + 3 * k;
        return V3{p[0], p[1], p[2]};
      };
      const double nan = __builtin_nan("");
      const int64_t g = a + r;
      const bool last = r == n - 1;
      const V3 N = at(r, 0), CA = at(r, 1), C = at(r, 2);
      double phi = nan, psi = nan, omega = nan, tau = nan, cac1n = nan, c1nca = nan;
      double d_cn = 0.0, d_nca = 0.0, d_cac = 0.0;
      if (r > 0) phi = bb_dihedral(at(r - 1, 2), N, CA, C);
      if (!last) {
        const V3 N1 = at(r + 1, 0), CA1 = at(r + 1, 1), C1 = at(r + 1, 2);
        psi = bb_dihedral(N, CA, C, N1);
        omega = bb_dihedral(CA, C, N1, CA1);
        tau = bb_angle(N1, CA1, C1);
        cac1n = bb_angle(CA, C, N1);
        c1nca = bb_angle(C, N1, CA1);
        d_cn = v_norm(v_sub(N1, C));
        d_nca = v_norm(v_sub(CA1, N1));
        d_cac = v_norm(v_sub(C1, CA1));
      }
      out[GEOBPE_COL_0C1N * R + g] = d_cn;
      out[GEOBPE_COL_NCA * R + g] = d_nca;
      out[GEOBPE_COL_CAC * R + g] = d_cac;
      out[GEOBPE_COL_PHI * R + g] = phi;
      out[GEOBPE_COL_PSI * R + g] = psi;
      out[GEOBPE_COL_OMEGA * R + g] = omega;
      out[GEOBPE_COL_TAU * R + g] = tau;
      out[GEOBPE_COL_CAC1N * R + g] = cac1n;
      out[GEOBPE_COL_C1NCA * R + g] = c1nca;
    }
  }
}

// ------------------------------------------------------------------ host: PDB reader
// amino-acid residue names accepted as backbone residues (the 20 standard ones and
// the common modified L-peptide-linking ones biotite's filter_amino_acids keeps)
inline bool pdb_amino_acid(const std::string& rn) {
  static const std::set<std::string> aa = {
      "ALA", "ARG", "ASN", "ASP", "CYS", "GLN", "GLU", "GLY", "HIS", "ILE", "LEU", "LYS", "MET", "PHE",
      "PRO", "SER", "THR", "TRP", "TYR", "VAL", "MSE", "SEC", "PYL", "SEP", "TPO", "PTR", "HYP", "MLY",
      "CSO", "CME", "KCX", "LLP", "CSD", "OCS", "M3L", "FME", "ASX", "GLX", "UNK"};
  return aa.count(rn) > 0;
}

inline std::string pdb_field(const std::string& s, size_t a, size_t b) {
  if (s.size() <= a) return "";
  std::string f = s.substr(a, std::min(b, s.size()) - a);
  size_t i = f.find_first_not_of(' '), j = f.find_last_not_of(' ');
  return i == std::string::npos ? "" : f.substr(i, j - i + 1);
}

// backbone of the first model: N, CA, C per residue in file order.  A residue
// missing one of the three is an error (biotite's dihedral_backbone raises
// BadStructureError; the reference then skips the file, angles_and_coords.py:92-94).
inline int pdb_backbone(const std::string& path, std::vector<double>& xyz, std::string& err) {
  std::ifstream f(path);
  if (!f) {
    err = "cannot open " + path;
    return -1;
  }
  struct Res {
    std::string key;
    bool has[3] = {false, false, false};
    double p[9];
  };
  std::vector<Res> res;
  std::string line;
  bool in_model = false;
  while (std::getline(f, line)) {
    const std::string rec = line.substr(0, 6);
    if (rec == "MODEL ") {
      if (in_model) break;
      in_model = true;
      continue;
    }
    if (rec == "ENDMDL") break;
    if ((rec != "ATOM  " && rec != "HETATM") || line.size() < 54) continue;
    const std::string name = pdb_field(line, 12, 16), resn = pdb_field(line, 17, 20);
    if (!pdb_amino_acid(resn)) continue;
    const int k = name == "N" ? 0 : name == "CA" ? 1 : name == "C" ? 2 : -1;
    const std::string key = line.substr(21, 1) + "|" + pdb_field(line, 22, 26) + "|" +
                            (line.size() > 26 ? line.substr(26, 1) : " ") + "|" + resn;
    if (res.empty() || res.back().key != key) {
      res.push_back(Res());
      res.back().key = key;
    }
    if (k < 0) continue;
    Res& r = res.back();
    if (r.has[k]) continue;  // the first alternate location only (get_structure's altloc="first")
    double x, y, z;
    try {
      x = std::stod(line.substr(30, 8));
      y = std::stod(line.substr(38, 8));
      z = std::stod(line.substr(46, 8));
    } catch (...) {
      err = "bad coordinates in " + path + ": " + line;
      return -1;
    }
    r.has[k] = true;
    r.p[3 * k] = x;
    r.p[3 * k + 1] = y;
    r.p[3 * k + 2] = z;
  }
  xyz.clear();
  for (const Res& r : res) {
    if (!(r.has[0] && r.has[1] && r.has[2])) {
      err = "residue " + r.key + " lacks a backbone atom (BadStructureError)";
      return -2;
    }
    xyz.insert(xyz.end(), r.p, r.p + 9);
  }
  return (int)res.size();
}

}  // namespace gb
