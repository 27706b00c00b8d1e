// frepr.cpp -- Python's repr(float) for rmsdkey.c, from std::to_chars' shortest round-trip
// digits (the same digits float.__repr__'s dtoa mode 0 picks; checked against repr on 3e5
// values, tests/test_rmsd_mode.py): fixed notation for a decimal point in (-4, 16], else
// d.ddde+XX with at least two exponent digits, ".0" after an integral fixed value.
// ~10x faster than PyOS_double_to_string, which dominated a key's cost; repeated values hit a cache.
#include <charconv>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>

static int repr_slow(double v, char* out) {
  char buf[40];
  auto r = std::to_chars(buf, buf + sizeof buf - 1, v, std::chars_format::scientific);
  *r.ptr = 0;
  const char* p = buf;
  int o = 0;
  if (*p == '-') {
    out[o++] = '-';
    p++;
  }
  char dig[32];
  int n = 0;
  while (*p && *p != 'e') {
    if (*p != '.') dig[n++] = *p;
    p++;
  }
  const int e = atoi(p + 1);
  if (n == 1 && dig[0] == '0') {
    memcpy(out + o, "0.0", 3);
    return o + 3;
  }
  const int decpt = e + 1;
  if (decpt > -4 && decpt <= 16) {
    if (decpt <= 0) {
      out[o++] = '0';
      out[o++] = '.';
      for (int i = 0; i < -decpt; i++) out[o++] = '0';
      memcpy(out + o, dig, n);
      o += n;
    } else if (decpt >= n) {
      memcpy(out + o, dig, n);
      o += n;
      for (int i = 0; i < decpt - n; i++) out[o++] = '0';
      out[o++] = '.';
      out[o++] = '0';
    } else {
      memcpy(out + o, dig, decpt);
      o += decpt;
      out[o++] = '.';
      memcpy(out + o, dig + decpt, n - decpt);
      o += n - decpt;
    }
  } else {
    out[o++] = dig[0];
    if (n > 1) {
      out[o++] = '.';
      memcpy(out + o, dig + 1, n - 1);
      o += n - 1;
    }
    const int x = decpt - 1;
    o += snprintf(out + o, 8, "e%c%02d", x < 0 ? '-' : '+', x < 0 ? -x : x);
  }
  return o;
}

// A key repeats the same values over and over (in the RMSD mode the chains carry their medoids'
// geometry): a direct-mapped cache of the last repr per slot, keyed by the double's bits.  The
// callers hold the GIL, so one table serves every call.
namespace {
struct Ent {
  uint64_t bits;
  uint8_t n;
  char s[31];
};
Ent g_cache[1 << 16];
}  // namespace

extern "C" int geobpe_py_repr(double v, char* out) {  // out: >= 32 bytes; returns the length
  uint64_t b;
  memcpy(&b, &v, 8);
  Ent& e = g_cache[(b * 0x9E3779B97F4A7C15ULL) >> 48];
  if (e.n && e.bits == b) {
    memcpy(out, e.s, e.n);
    return e.n;
  }
  const int n = repr_slow(v, out);
  if (n <= (int)sizeof e.s) {
    e.bits = b;
    e.n = (uint8_t)n;
    memcpy(e.s, out, n);
  }
  return n;
}
