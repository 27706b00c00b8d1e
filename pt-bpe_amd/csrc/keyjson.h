// keyjson.h -- the reference's pair-key string and its ordering (host side).
//
// The reference keys every adjacent-token pair by
//   json.dumps(geo, sort_keys=True)            (BPE.hash_geo, foldingdiff/bpe.py:1147-1149)
// of the quantised geometry of the span (compute_geo_key, bpe.py:1192-1299), and
// breaks count ties by the smallest such string (SortedDict over
// (True, -count, key), bpe.py:1469-1471).  For the scoped mode (std_bonds, one
// bin grid) the string is a pure function of the span's CONTENT: the residue
// symbols R (tau*B^2 + cac1n*B + psi, or B^3 + tau for a chain's last residue)
// and junction symbols G (omega*B^2 + cnca*B + phi) -- SURVEY.md Appendix A.
// This header renders that string from a content so the tie-break can compare
// real reference strings.
#pragma once
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

namespace geobpe {

// content: R0 G0 R1 G1 ... R_{r-1}  (2r-1 symbols)
// limit > 0: stop once at least `limit` characters are produced (prefix).
inline void render_key(const int32_t* s, int64_t nsym, int32_t B, std::string& out, size_t limit = 0) {
  const int64_t r = (nsym + 1) / 2;
  const int32_t B2 = B * B, B3 = B2 * B;
  const int lam = s[nsym - 1] >= B3 ? 1 : 0;
  out.clear();
  char t[16];
  auto num = [&](int32_t v) {
    int m = snprintf(t, sizeof t, "%d", v);
    out.append(t, m);
  };
  auto zeros = [&](const char* name, int64_t cnt) {
    out += '"';
    out += name;
    out += "\": [";
    for (int64_t q = 0; q < cnt; q++) {
      if (q) out += ", ";
      out += '0';
    }
    out += ']';
  };
#define GEOBPE_STOP \
  if (limit && out.size() >= limit) return
  out += '{';
  zeros("0C:1N", r - lam);
  GEOBPE_STOP;
  out += ", \"C:1N:1CA\": [";
  for (int64_t j = 0; j < r - 1; j++) {
    if (j) out += ", ";
    num(s[2 * j + 1] / B % B);
    GEOBPE_STOP;
  }
  out += "], ";
  zeros("CA:C", r);
  out += ", \"CA:C:1N\": [";
  for (int64_t j = 0; j < r - lam; j++) {
    if (j) out += ", ";
    num(s[2 * j] / B % B);
    GEOBPE_STOP;
  }
  out += "], ";
  zeros("N:CA", r);
  GEOBPE_STOP;
  out += ", \"omega\": [";
  for (int64_t j = 0; j < r - 1; j++) {
    if (j) out += ", ";
    num(s[2 * j + 1] / B2);
  }
  out += "], \"phi\": [";
  for (int64_t j = 0; j < r - 1; j++) {
    if (j) out += ", ";
    num(s[2 * j + 1] % B);
  }
  out += "], \"psi\": [";
  for (int64_t j = 0; j < r - lam; j++) {
    if (j) out += ", ";
    num(s[2 * j] % B);
  }
  out += "], \"tau\": [";
  for (int64_t j = 0; j < r; j++) {
    if (j) out += ", ";
    const int32_t x = s[2 * j];
    num(x >= B3 ? x - B3 : x / B2);
  }
  out += "]}";
#undef GEOBPE_STOP
}

}  // namespace geobpe
