// geobpe.hip -- MI355X (gfx950) GeoBPE merge loop: HIP kernels + the C-ABI
// declared in include/geobpe.h.
//
// Replaces the Python/dict hot path of foldingdiff/bpe.py (BPE.initialize /
// bin / step / quantize).  Integer work only: no
// MFMA.  Design:
//
//  * Residue-indexed token state in HBM (one int32 per residue per array):
//      tid   token id at a token's first residue, -1 elsewhere
//      tlen  residues covered by the token
//      tprev first residue of the previous token in the chain (-1 at chain start)
//      pk    dense key id of the pair (token, next token), -1 if none / dead
//    A token's content (R G R ... R symbols) is identified by a 2x61-bit
//    polynomial hash, so the pair key of (X, g, Y) is computed from (hX, g, hY,
//    |Y|) without touching the residues: that is the split-invariant, content-
//    keyed pair key of compute_geo_key (bpe.py:1192-1299).
//  * A global key dictionary: open-addressing table (64-bit probe key, CAS
//    claim) -> dense key id; per dense key: hash, length, a representative
//    (idL, g, idR) and the live occurrence count.
//  * bin(): every adjacent pair is hashed and inserted (k_pairs_all), new keys
//    get dense ids (k_assign), counts are accumulated with LDS-staged
//    per-workgroup partial counts flushed by global atomics (k_finalize).
//  * step(): device argmax over the dense counts (k_argmax + k_cands; ties
//    resolved on the host with the real reference key strings), k_mark scans
//    pk for the winner and walks each maximal run of matches applying the
//    greedy left-to-right rule (bpe.py:1888-1916), compacting the merge list
//    with a wavefront ballot / prefix sum, and k_apply rewrites the tokens and
//    issues the incremental count deltas (bpe.py:1924-2138).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/geobpe.h"
#include "keyjson.h"

typedef unsigned long long u64;

namespace {

constexpr u64 M61 = (1ULL << 61) - 1;
constexpr u64 HP1 = 0x0A3B5C7D9E1F2437ULL % M61;  // hash bases (< M61)
constexpr u64 HP2 = 0x13579BDF2468ACE1ULL % M61;
constexpr u64 KMIX = 0x9E3779B97F4A7C15ULL;
constexpr double TWO_PI = 6.283185307179586;  // 2*np.pi
constexpr int BLOCK = 256;
constexpr int AGG = 2048;  // LDS partial-count slots per workgroup

// ------------------------------------------------------------------ device structs
struct State {
  // persistent
  int64_t U;         // dense keys allocated
  int64_t err_code;  // first error (GEOBPE_E*)
  int64_t err_pos;
  int64_t epoch;     // delta-touch epoch (multi-rank)
  // per-iteration (zeroed by memset from here on)
  int32_t maxc;
  int32_t pad0;
  int64_t ncand;
  int64_t nL;
  int64_t nnew_pairs;
  int64_t nnew_slots;
  int64_t ntouched;
  int64_t nmismatch;
};
constexpr size_t STATE_ITER_OFF = offsetof(State, maxc);

struct Cand {
  int32_t d, idL, g, idR;
};
struct LEntry {
  int32_t a, p, b, c;
};
struct NewPair {
  int32_t target;  // residue whose pk receives the key (-1: none)
  int32_t slot;    // table slot
  int32_t len;     // residues of the pair content
  int32_t delta;   // count contribution
  u64 h1, h2;
};
struct NewSlot {
  int32_t slot, len;
  int32_t idL, g, idR, pad;
  u64 h1, h2;
};
struct DeltaRec {  // 40 bytes, exchanged between ranks
  u64 h1, h2;
  int32_t len, idL, g, idR, delta, pad;
};
static_assert(sizeof(DeltaRec) == 40, "delta record layout");

struct Dev {
  // corpus
  int64_t R, nrows;
  int32_t B, B2, B3, pad;
  const int64_t* row_off;
  int32_t *rsym, *gsym;
  // tokens
  int32_t *tid, *tlen, *tprev, *pk, *role;
  // vocab
  u64 *vh1, *vh2;
  int32_t* vlen;
  int64_t KC;
  // powers
  const u64 *pw1, *pw2;
  int64_t pwn;
  // key table
  u64* ht_key;
  int32_t* ht_dense;
  int64_t HC;
  int32_t ht_shift;
  int32_t pad2;
  // dense keys
  u64 *kh1, *kh2;
  int32_t *klen, *krep, *count, *dcount, *touch, *touched, *scratch;
  int64_t UC;
  // work lists
  LEntry* L;
  int64_t Lcap;
  NewPair* np;
  NewSlot* ns;
  int64_t npcap;
  Cand* cand;
  int64_t candcap;
  State* st;
};

// ------------------------------------------------------------------ device helpers
__host__ __device__ inline u64 mulmod61(u64 a, u64 b) {
#if defined(__HIP_DEVICE_COMPILE__)
  u64 lo = a * b;
  u64 hi = __umul64hi(a, b);
#else
  unsigned __int128 p = (unsigned __int128)a * b;
  u64 lo = (u64)p, hi = (u64)(p >> 64);
#endif
  u64 r = (lo & M61) + ((lo >> 61) | (hi << 3));
  r = (r & M61) + (r >> 61);
  return r >= M61 ? r - M61 : r;
}
__host__ __device__ inline u64 addmod61(u64 a, u64 b) {
  u64 r = a + b;
  return r >= M61 ? r - M61 : r;
}

// hash of content X ++ [g] ++ Y given the hashes of X and Y and |Y| residues
__device__ inline void combine(const Dev& D, u64 x1, u64 x2, int32_t g, u64 y1, u64 y2, int32_t ylen, u64& o1,
                               u64& o2) {
  const int64_t ny = 2 * (int64_t)ylen - 1;
  const u64 gg = (u64)(g + 1);
  o1 = addmod61(addmod61(mulmod61(x1, D.pw1[ny + 1]), mulmod61(gg, D.pw1[ny])), y1);
  o2 = addmod61(addmod61(mulmod61(x2, D.pw2[ny + 1]), mulmod61(gg, D.pw2[ny])), y2);
}

__device__ inline u64 probe_key(u64 h1, u64 h2, int32_t len) {
  u64 k = (h1 * KMIX) ^ (h2 + ((u64)len << 40)) ^ (h2 >> 29);
  return k ? k : 1;
}

__device__ inline void set_error(const Dev& D, int64_t code, int64_t pos) {
  unsigned long long* p = (unsigned long long*)&D.st->err_code;
  if (atomicCAS(p, 0ULL, (unsigned long long)code) == 0ULL) D.st->err_pos = pos;
}

// Python/numpy (v + 2*pi) % (2*pi) for float64 (float_rem / npy_divmod)
__device__ inline double wrap2pi(double v) {
  const double a = v + TWO_PI;
  double m;
  if (a >= 0.0 && a < TWO_PI)
    m = a;
  else if (a >= TWO_PI && a < 2.0 * TWO_PI)
    m = a - TWO_PI;  // exact (Sterbenz)
  else
    m = fmod(a, TWO_PI);
  if (m != 0.0) {
    if (m < 0.0) m += TWO_PI;
  } else {
    m = 0.0;
  }
  return m;
}

// BPE.get_ind (bpe.py:1164-1189); returns -1 where the reference raises ValueError
__device__ inline int32_t get_ind(const double* e, int32_t B, double v) {
  int32_t lo = 0, hi = B;  // bisect_right over the B left edges e[0..B-1]
  while (lo < hi) {
    int32_t mid = (lo + hi) >> 1;
    if (v < e[mid])
      hi = mid;
    else
      lo = mid + 1;
  }
  const int32_t ind = lo - 1;
  if (ind < 0) return -1;
  const double s = e[ind], t = e[ind + 1];
  if (ind == B - 1 && v == t) return ind;
  if (s <= v && v < t) return ind;
  return -1;
}

__device__ inline int wave_lane() { return threadIdx.x & 63; }

// exclusive prefix sum across the 64-lane wavefront
__device__ inline int32_t wave_excl_scan(int32_t v, int32_t& total) {
  int32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int32_t y = __shfl_up(x, o, 64);
    if (wave_lane() >= o) x += y;
  }
  total = __shfl(x, 63, 64);
  return x - v;
}

__device__ inline int32_t wave_max(int32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

// wave-aggregated append: returns this lane's index (or -1 when !want)
__device__ inline int64_t wave_append(bool want, int64_t* counter) {
  const u64 mask = __ballot(want);
  if (!mask) return -1;
  const int lane = wave_lane();
  const int leader = __ffsll((long long)mask) - 1;
  int64_t base = 0;
  if (lane == leader) base = atomicAdd((unsigned long long*)counter, (unsigned long long)__popcll(mask));
  base = __shfl(base, leader, 64);
  if (!want) return -1;
  return base + __popcll(mask & ((1ULL << lane) - 1ULL));
}

// count update target: global counts, or the rank-local delta + touched list
__device__ inline void global_add(const Dev& D, int32_t d, int32_t v, bool to_delta) {
  if (!to_delta) {
    atomicAdd(&D.count[d], v);
    return;
  }
  atomicAdd(&D.dcount[d], v);
  const int32_t ep = (int32_t)D.st->epoch;
  if (atomicExch(&D.touch[d], ep) != ep) {
    const int64_t j = atomicAdd((unsigned long long*)&D.st->ntouched, 1ULL);
    D.touched[j] = d;
  }
}

// LDS-staged per-workgroup partial counts
struct Agg {
  int32_t key[AGG];
  int32_t val[AGG];
};
__device__ inline void agg_init(Agg& s) {
  for (int i = threadIdx.x; i < AGG; i += blockDim.x) {
    s.key[i] = -1;
    s.val[i] = 0;
  }
  __syncthreads();
}
__device__ inline void agg_add(Agg& s, const Dev& D, int32_t d, int32_t v, bool to_delta) {
  uint32_t h = ((uint32_t)d * 2654435761u) >> 21;  // 11 bits
#pragma unroll 1
  for (int probe = 0; probe < 8; probe++) {
    const int32_t k = s.key[h];
    if (k == d) {
      atomicAdd(&s.val[h], v);
      return;
    }
    if (k == -1) {
      const int32_t old = atomicCAS(&s.key[h], -1, d);
      if (old == -1 || old == d) {
        atomicAdd(&s.val[h], v);
        return;
      }
    }
    h = (h + 1) & (AGG - 1);
  }
  global_add(D, d, v, to_delta);
}
__device__ inline void agg_flush(Agg& s, const Dev& D, bool to_delta) {
  __syncthreads();
  for (int i = threadIdx.x; i < AGG; i += blockDim.x) {
    const int32_t k = s.key[i];
    if (k >= 0 && s.val[i] != 0) global_add(D, k, s.val[i], to_delta);
  }
}

// find-or-claim the table slot of a key; new keys are appended to the slot list
__device__ inline int32_t ht_insert(const Dev& D, u64 h1, u64 h2, int32_t len, int32_t idL, int32_t g,
                                    int32_t idR) {
  const u64 k = probe_key(h1, h2, len);
  u64 s = (k * 0xD6E8FEB86659FD93ULL) >> D.ht_shift;
  const u64 mask = (u64)D.HC - 1;
  for (int64_t probe = 0; probe < D.HC; probe++) {
    const u64 cur = D.ht_key[s];
    if (cur == k) return (int32_t)s;
    if (cur == 0) {
      const u64 old = atomicCAS((unsigned long long*)&D.ht_key[s], 0ULL, (unsigned long long)k);
      if (old == 0) {
        const int64_t j = atomicAdd((unsigned long long*)&D.st->nnew_slots, 1ULL);
        if (j < D.npcap) {
          NewSlot e;
          e.slot = (int32_t)s;
          e.len = len;
          e.idL = idL;
          e.g = g;
          e.idR = idR;
          e.pad = 0;
          e.h1 = h1;
          e.h2 = h2;
          D.ns[j] = e;
        } else {
          set_error(D, GEOBPE_ECAPACITY, j);
        }
        return (int32_t)s;
      }
      if (old == k) return (int32_t)s;
    }
    s = (s + 1) & mask;
  }
  set_error(D, GEOBPE_ECAPACITY, -2);
  return -1;
}

__device__ inline void push_pair(const Dev& D, int32_t target, int32_t slot, int32_t len, int32_t delta, u64 h1,
                                 u64 h2) {
  const int64_t j = atomicAdd((unsigned long long*)&D.st->nnew_pairs, 1ULL);
  if (j >= D.npcap) {
    set_error(D, GEOBPE_ECAPACITY, -3);
    return;
  }
  NewPair e;
  e.target = target;
  e.slot = slot;
  e.len = len;
  e.delta = delta;
  e.h1 = h1;
  e.h2 = h2;
  D.np[j] = e;
}

// ------------------------------------------------------------------ kernels: prologue
// threshold types -> column index
__constant__ int32_t c_type_col[GEOBPE_NTYPES] = {GEOBPE_COL_TAU,   GEOBPE_COL_CAC1N, GEOBPE_COL_C1NCA,
                                                  GEOBPE_COL_PSI,   GEOBPE_COL_OMEGA, GEOBPE_COL_PHI};

struct Cols {
  const double* c[9];
};

// per (block, type) min / max / count of the wrapped non-NaN non-zero values
__global__ __launch_bounds__(BLOCK) void k_range(Cols cols, int64_t R, double* part) {
  const int t = blockIdx.y;
  const double* x = cols.c[c_type_col[t]];
  double mn = INFINITY, mx = -INFINITY;
  int64_t cnt = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < R; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = x[i];
    if (v == v && v != 0.0) {
      const double w = wrap2pi(v);
      mn = fmin(mn, w);
      mx = fmax(mx, w);
      cnt++;
    }
  }
  __shared__ double smn[BLOCK], smx[BLOCK];
  __shared__ int64_t scn[BLOCK];
  smn[threadIdx.x] = mn;
  smx[threadIdx.x] = mx;
  scn[threadIdx.x] = cnt;
  __syncthreads();
  for (int o = BLOCK / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      smn[threadIdx.x] = fmin(smn[threadIdx.x], smn[threadIdx.x + o]);
      smx[threadIdx.x] = fmax(smx[threadIdx.x], smx[threadIdx.x + o]);
      scn[threadIdx.x] += scn[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double* p = part + ((int64_t)t * gridDim.x + blockIdx.x) * 3;
    p[0] = smn[0];
    p[1] = smx[0];
    p[2] = (double)scn[0];
  }
}

// residue / junction symbols (tokenizer.py:131-167 index maps)
__global__ __launch_bounds__(64) void k_quantize(Dev D, Cols cols, const double* edges, double init_tau) {
  const int32_t B = D.B;
  const double* eT = edges + 0 * (B + 1);
  const double* eA = edges + 1 * (B + 1);
  const double* eC = edges + 2 * (B + 1);
  const double* eP = edges + 3 * (B + 1);
  const double* eO = edges + 4 * (B + 1);
  const double* eF = edges + 5 * (B + 1);
  const double* tau = cols.c[GEOBPE_COL_TAU];
  const double* cac1n = cols.c[GEOBPE_COL_CAC1N];
  const double* c1nca = cols.c[GEOBPE_COL_C1NCA];
  const double* psi = cols.c[GEOBPE_COL_PSI];
  const double* omega = cols.c[GEOBPE_COL_OMEGA];
  const double* phi = cols.c[GEOBPE_COL_PHI];
  for (int64_t r = blockIdx.x; r < D.nrows; r += gridDim.x) {
    const int64_t a = D.row_off[r], b = D.row_off[r + 1];
    for (int64_t g = a + threadIdx.x; g < b; g += blockDim.x) {
      const bool last = (g == b - 1);
      const double ts = (g == a) ? init_tau : tau[g - 1];  // tau_j = df.tau[j-1]
      const int32_t tb = get_ind(eT, B, wrap2pi(ts));
      int32_t rs, gs = -1;
      bool bad = tb < 0;
      if (!last) {
        const int32_t ab = get_ind(eA, B, wrap2pi(cac1n[g]));
        const int32_t pb = get_ind(eP, B, wrap2pi(psi[g]));
        const int32_t ob = get_ind(eO, B, wrap2pi(omega[g]));
        const int32_t cb = get_ind(eC, B, wrap2pi(c1nca[g]));
        const int32_t fb = get_ind(eF, B, wrap2pi(phi[g + 1]));
        bad = bad || ab < 0 || pb < 0 || ob < 0 || cb < 0 || fb < 0;
        rs = tb * D.B2 + ab * B + pb;
        gs = ob * D.B2 + cb * B + fb;
      } else {
        rs = D.B3 + tb;
      }
      if (bad) {
        set_error(D, GEOBPE_EVALUE, g);
        rs = last ? D.B3 : 0;
        gs = last ? -1 : 0;
      }
      D.rsym[g] = rs;
      D.gsym[g] = gs;
    }
  }
}

// first appearance of every residue symbol (label order of bpe.py:236-246)
__global__ __launch_bounds__(BLOCK) void k_first(Dev D, int64_t row_base, u64* first, int32_t S, int use_lds) {
  extern __shared__ u64 sfirst[];
  if (use_lds) {
    for (int i = threadIdx.x; i < S; i += blockDim.x) sfirst[i] = ~0ULL;
    __syncthreads();
  }
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < D.R; g += (int64_t)gridDim.x * blockDim.x) {
    const int32_t s = D.rsym[g];
    if (use_lds)
      atomicMin(&sfirst[s], (u64)(g + row_base));
    else
      atomicMin((unsigned long long*)&first[s], (unsigned long long)(g + row_base));
  }
  if (use_lds) {
    __syncthreads();
    for (int i = threadIdx.x; i < S; i += blockDim.x)
      if (sfirst[i] != ~0ULL) atomicMin((unsigned long long*)&first[i], (unsigned long long)sfirst[i]);
  }
}

__global__ __launch_bounds__(64) void k_init_tokens(Dev D, const int32_t* label_of_sym) {
  for (int64_t r = blockIdx.x; r < D.nrows; r += gridDim.x) {
    const int64_t a = D.row_off[r], b = D.row_off[r + 1];
    for (int64_t g = a + threadIdx.x; g < b; g += blockDim.x) {
      D.tid[g] = label_of_sym[D.rsym[g]];
      D.tlen[g] = 1;
      D.tprev[g] = (g == a) ? -1 : (int32_t)(g - 1);
      D.pk[g] = -1;
      D.role[g] = 0;
    }
  }
}

// ------------------------------------------------------------------ kernels: histogram
// every live adjacent pair -> content hash -> key slot (BPE.bin, bpe.py:1431-1474)
__global__ __launch_bounds__(BLOCK) void k_pairs_all(Dev D) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < D.R; g += (int64_t)gridDim.x * blockDim.x) {
    const int32_t L = D.tid[g];
    if (L < 0) continue;
    const int32_t e = (int32_t)g + D.tlen[g] - 1;
    if (D.rsym[e] >= D.B3) continue;  // last token of its chain
    const int32_t Rr = D.tid[e + 1];
    const int32_t gl = D.gsym[e];
    const int32_t ylen = D.vlen[Rr];
    u64 h1, h2;
    combine(D, D.vh1[L], D.vh2[L], gl, D.vh1[Rr], D.vh2[Rr], ylen, h1, h2);
    const int32_t len = D.vlen[L] + ylen;
    const int32_t slot = ht_insert(D, h1, h2, len, L, gl, Rr);
    if (slot >= 0) push_pair(D, (int32_t)g, slot, len, 1, h1, h2);
  }
}

// dense ids for the keys claimed since the last commit
__global__ __launch_bounds__(BLOCK) void k_assign(Dev D) {
  const int64_t n = D.st->nnew_slots;
  const int64_t U = D.st->U;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    const NewSlot e = D.ns[j];
    const int64_t d = U + j;
    if (d >= D.UC) {
      set_error(D, GEOBPE_ECAPACITY, -4);
      continue;
    }
    D.ht_dense[e.slot] = (int32_t)d;
    D.kh1[d] = e.h1;
    D.kh2[d] = e.h2;
    D.klen[d] = e.len;
    D.krep[3 * d + 0] = e.idL;
    D.krep[3 * d + 1] = e.g;
    D.krep[3 * d + 2] = e.idR;
    D.count[d] = 0;
    if (D.dcount) {
      D.dcount[d] = 0;
      D.touch[d] = -1;
    }
  }
}

// pair -> dense key id into pk, and the counts (LDS-staged partial counts)
__global__ __launch_bounds__(BLOCK) void k_finalize(Dev D, int to_delta) {
  __shared__ Agg agg;
  agg_init(agg);
  if (blockIdx.x == 0 && threadIdx.x == 0) D.st->U += D.st->nnew_slots;
  const int64_t n = D.st->nnew_pairs;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    const NewPair e = D.np[j];
    const int32_t d = D.ht_dense[e.slot];
    if (d < 0 || D.kh1[d] != e.h1 || D.kh2[d] != e.h2 || D.klen[d] != e.len) {
      set_error(D, GEOBPE_EHASH, j);
      continue;
    }
    if (e.target >= 0) D.pk[e.target] = d;
    agg_add(agg, D, d, e.delta, to_delta != 0);
  }
  agg_flush(agg, D, to_delta != 0);
}

// ------------------------------------------------------------------ kernels: step
__global__ __launch_bounds__(BLOCK) void k_argmax(Dev D) {
  const int64_t U = D.st->U;
  int32_t m = 0;
  for (int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; d < U; d += (int64_t)gridDim.x * blockDim.x)
    m = max(m, D.count[d]);
  m = wave_max(m);
  __shared__ int32_t sm[BLOCK / 64];
  if (wave_lane() == 0) sm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t x = sm[0];
    for (int i = 1; i < BLOCK / 64; i++) x = max(x, sm[i]);
    if (x > 0) atomicMax(&D.st->maxc, x);
  }
}

__global__ __launch_bounds__(BLOCK) void k_cands(Dev D) {
  const int64_t U = D.st->U;
  const int32_t mc = D.st->maxc;
  if (mc <= 0) return;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t Ur = (U + 63) & ~63LL;
  for (int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; d - threadIdx.x % 64 < Ur; d += stride) {
    const bool hit = d < U && D.count[d] == mc;
    const int64_t j = wave_append(hit, &D.st->ncand);
    if (hit && j < D.candcap) {
      Cand c;
      c.d = (int32_t)d;
      c.idL = D.krep[3 * d];
      c.g = D.krep[3 * d + 1];
      c.idR = D.krep[3 * d + 2];
      D.cand[j] = c;
    }
  }
}

// walk one maximal run of winner matches starting at token h (greedy left to
// right, bpe.py:1888-1916): merges h, skips the next pair, merges the one
// after if the run continues, ...
__device__ inline int32_t walk_run(const Dev& D, int32_t h, int32_t W, int32_t tag, int64_t out) {
  int32_t t = h, p = D.tprev[h], n = 0;
  for (;;) {
    const int32_t b = t + D.tlen[t];
    const int32_t pkb = D.pk[b];
    const int32_t c = pkb >= 0 ? b + D.tlen[b] : -1;
    if (out >= 0) {
      LEntry e;
      e.a = t;
      e.p = p;
      e.b = b;
      e.c = c;
      D.L[out + n] = e;
      D.role[t] = (tag << 2) | 1;
      D.role[b] = (tag << 2) | 2;
    }
    n++;
    if (pkb != W) break;
    if (D.pk[c] != W) break;
    p = b;
    t = c;
  }
  return n;
}

// scan pk for the winner (4 residues per lane, int4 loads), find run starts,
// compact the merge list with a wave prefix sum
__global__ __launch_bounds__(BLOCK) void k_mark(Dev D, int32_t W, int32_t tag) {
  const int64_t n4 = (D.R + 3) / 4;
  const int4* pk4 = reinterpret_cast<const int4*>(D.pk);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4r = (n4 + 63) & ~63LL;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i - threadIdx.x % 64 < n4r; i += stride) {
    int32_t starts[4];
    int ns = 0;
    if (i < n4) {
      const int4 v = pk4[i];
      const int32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; q++) {
        if (vv[q] == W) {
          const int32_t g = (int32_t)(4 * i + q);
          const int32_t p = D.tprev[g];
          if (p < 0 || D.pk[p] != W) starts[ns++] = g;
        }
      }
    }
    const bool any = __ballot(ns > 0) != 0ULL;
    if (!any) continue;
    int32_t cnt = 0;
    for (int q = 0; q < ns; q++) cnt += walk_run(D, starts[q], W, tag, -1);
    int32_t total;
    const int32_t off = wave_excl_scan(cnt, total);
    int64_t base = 0;
    if (wave_lane() == 0) base = atomicAdd((unsigned long long*)&D.st->nL, (unsigned long long)total);
    base = __shfl(base, 0, 64);
    if (base + total > D.Lcap) {
      if (wave_lane() == 0) set_error(D, GEOBPE_ECAPACITY, -5);
      continue;
    }
    int64_t o = base + off;
    for (int q = 0; q < ns; q++) o += walk_run(D, starts[q], W, tag, o);
  }
}

// rewrite every merged occurrence and issue the count deltas (bpe.py:1924-2014)
__global__ __launch_bounds__(BLOCK) void k_apply(Dev D, int32_t W, int32_t nid, int32_t tag, int to_delta) {
  __shared__ Agg agg;
  agg_init(agg);
  const int64_t n = D.st->nL;
  const u64 w1 = D.kh1[W], w2 = D.kh2[W];
  const int32_t wl = D.klen[W];
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // _tokens[n] = json.loads(key)
    D.vh1[nid] = w1;
    D.vh2[nid] = w2;
    D.vlen[nid] = wl;
  }
  const int32_t tagR = (tag << 2) | 2, tagL = (tag << 2) | 1;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    const LEntry e = D.L[j];
    const int32_t pkb = D.pk[e.b];
    agg_add(agg, D, W, -1, to_delta != 0);                       // step 1
    if (pkb >= 0) agg_add(agg, D, pkb, -1, to_delta != 0);       // step 4 (right pair)
    const bool pN = e.p >= 0 && D.role[e.p] != tagR;
    if (pN) agg_add(agg, D, D.pk[e.p], -1, to_delta != 0);       // step 3 (left pair)
    D.tid[e.a] = nid;                                            // step 2
    D.tlen[e.a] = wl;
    D.tid[e.b] = -1;
    D.pk[e.b] = -1;
    if (e.c >= 0) D.tprev[e.c] = e.a;
    if (pN) {                                                    // step 5 (new left pair)
      const int32_t L = D.tid[e.p];
      const int32_t gl = D.gsym[e.a - 1];
      u64 h1, h2;
      combine(D, D.vh1[L], D.vh2[L], gl, w1, w2, wl, h1, h2);
      const int32_t len = D.vlen[L] + wl;
      const int32_t slot = ht_insert(D, h1, h2, len, L, gl, nid);
      if (slot >= 0) push_pair(D, e.p, slot, len, 1, h1, h2);
    }
    if (e.c >= 0) {                                              // step 5 (new right pair)
      const bool cL = D.role[e.c] == tagL;
      const int32_t idr = cL ? nid : D.tid[e.c];
      const u64 r1 = cL ? w1 : D.vh1[idr], r2 = cL ? w2 : D.vh2[idr];
      const int32_t rl = cL ? wl : D.vlen[idr];
      const int32_t gl = D.gsym[e.a + wl - 1];
      u64 h1, h2;
      combine(D, w1, w2, gl, r1, r2, rl, h1, h2);
      const int32_t slot = ht_insert(D, h1, h2, wl + rl, nid, gl, idr);
      if (slot >= 0) push_pair(D, e.a, slot, wl + rl, 1, h1, h2);
    } else {
      D.pk[e.a] = -1;
    }
  }
  agg_flush(agg, D, to_delta != 0);
}

// ------------------------------------------------------------------ kernels: multi-rank deltas
__global__ __launch_bounds__(BLOCK) void k_export(Dev D, DeltaRec* out, int64_t cap) {
  const int64_t n = D.st->ntouched;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n && j < cap;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int32_t d = D.touched[j];
    DeltaRec r;
    r.h1 = D.kh1[d];
    r.h2 = D.kh2[d];
    r.len = D.klen[d];
    r.idL = D.krep[3 * d];
    r.g = D.krep[3 * d + 1];
    r.idR = D.krep[3 * d + 2];
    r.delta = D.dcount[d];
    r.pad = 0;
    D.dcount[d] = 0;
    out[j] = r;
  }
}

__global__ __launch_bounds__(BLOCK) void k_import(Dev D, const DeltaRec* in, int64_t n) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    const DeltaRec r = in[j];
    if (r.delta == 0) continue;
    const int32_t slot = ht_insert(D, r.h1, r.h2, r.len, r.idL, r.g, r.idR);
    if (slot >= 0) push_pair(D, -1, slot, r.len, r.delta, r.h1, r.h2);
  }
}

// ------------------------------------------------------------------ kernels: exports / checks
__global__ __launch_bounds__(BLOCK) void k_row_ntok(Dev D, int64_t* ntok) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < D.nrows; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = D.row_off[r], b = D.row_off[r + 1];
    int64_t n = 0;
    for (int64_t g = a; g < b; g += D.tlen[g]) n++;
    ntok[r] = n;
  }
}

__global__ __launch_bounds__(BLOCK) void k_row_seg(Dev D, const int64_t* tok_off, int32_t* start, int32_t* id) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < D.nrows; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = D.row_off[r], b = D.row_off[r + 1];
    int64_t t = tok_off[r];
    for (int64_t g = a; g < b; g += D.tlen[g]) {
      start[t] = (int32_t)(g - a);
      id[t] = D.tid[g];
      t++;
    }
  }
}

// quantize(tokenize()) per row: id, then K+B+omega, K+2B+phi, K+cnca
__global__ __launch_bounds__(BLOCK) void k_row_encode(Dev D, const int64_t* id_off, int32_t* ids, int32_t K) {
  const int32_t B = D.B;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < D.nrows; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = D.row_off[r], b = D.row_off[r + 1];
    int64_t t = id_off[r];
    for (int64_t g = a; g < b;) {
      const int64_t e = g + D.tlen[g] - 1;
      ids[t++] = D.tid[g];
      if (e + 1 < b) {
        const int32_t gs = D.gsym[e];
        ids[t++] = K + B + gs / D.B2;
        ids[t++] = K + 2 * B + gs % B;
        ids[t++] = K + gs / B % B;
      }
      g = e + 1;
    }
  }
}

__global__ __launch_bounds__(BLOCK) void k_recount(Dev D) {
  __shared__ Agg agg;
  agg_init(agg);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < D.R; g += stride) {
    const int32_t d = D.pk[g];
    if (d >= 0) {
      uint32_t h = ((uint32_t)d * 2654435761u) >> 21;
      bool done = false;
      for (int probe = 0; probe < 8 && !done; probe++) {
        const int32_t k = agg.key[h];
        if (k == d) {
          atomicAdd(&agg.val[h], 1);
          done = true;
        } else if (k == -1) {
          const int32_t old = atomicCAS(&agg.key[h], -1, d);
          if (old == -1 || old == d) {
            atomicAdd(&agg.val[h], 1);
            done = true;
          }
        }
        h = (h + 1) & (AGG - 1);
      }
      if (!done) atomicAdd(&D.scratch[d], 1);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < AGG; i += blockDim.x)
    if (agg.key[i] >= 0) atomicAdd(&D.scratch[agg.key[i]], agg.val[i]);
}

__global__ __launch_bounds__(BLOCK) void k_compare(Dev D) {
  const int64_t U = D.st->U;
  for (int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; d < U; d += (int64_t)gridDim.x * blockDim.x)
    if (D.scratch[d] != D.count[d]) atomicAdd((unsigned long long*)&D.st->nmismatch, 1ULL);
}

}  // namespace

// ====================================================================== host side
struct geobpe_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::string err;
  int64_t max_vocab = 0;
  // corpus
  int64_t nrows = 0, R = 0, Lmax = 1;
  int32_t B = 0;
  std::vector<int64_t> row_off;
  double* d_cols[9] = {nullptr};
  int64_t* d_row_off = nullptr;
  // device arrays
  Dev D{};
  void* allocs[64] = {nullptr};
  int nallocs = 0;
  State* h_state = nullptr;  // pinned
  Cand* h_cand = nullptr;    // pinned
  bool keys_ready = false;
  bool distributed = false;
  int64_t global_residues = 0;
  int32_t tag = 0;
  // host vocab (content per token id)
  std::vector<std::vector<int32_t>> vocab;
  int32_t K0 = 0;
  int grid = 2048;
  // pending selection (split step)
  int32_t sel_W = -1, sel_new = -1, sel_count = 0;
  // profiling
  bool prof = false;
  std::map<std::string, std::pair<double, int64_t>> ktime;
  struct Pend {
    std::string name;
    hipEvent_t a, b;
  };
  std::vector<Pend> pending;
  std::vector<hipEvent_t> evpool, evall;
};

namespace {

hipEvent_t take_event(geobpe_ctx* c) {
  if (c->evpool.empty()) {
    hipEvent_t e;
    hipEventCreate(&e);
    c->evall.push_back(e);
    return e;
  }
  hipEvent_t e = c->evpool.back();
  c->evpool.pop_back();
  return e;
}

int fail(geobpe_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  c->err = buf;
  return code;
}

#define HIPCHK(c, x)                                                                         \
  do {                                                                                       \
    hipError_t _e = (x);                                                                     \
    if (_e != hipSuccess) return fail(c, GEOBPE_EHIP, "%s: %s", #x, hipGetErrorString(_e)); \
  } while (0)

template <class T>
int dalloc(geobpe_ctx* c, T** p, int64_t n) {
  if (n <= 0) n = 1;
  void* q = nullptr;
  hipError_t e = hipMalloc(&q, (size_t)n * sizeof(T));
  if (e != hipSuccess)
    return fail(c, GEOBPE_EHIP, "hipMalloc(%lld bytes): %s", (long long)(n * sizeof(T)), hipGetErrorString(e));
  c->allocs[c->nallocs++] = q;
  *p = (T*)q;
  return 0;
}

// Light per-kernel timing: HIP events recorded on the context stream around each
// launch, collected (one synchronize) only when geobpe_kernel_ms() is called.
struct Timed {
  geobpe_ctx* c;
  const char* name;
  hipEvent_t a = nullptr, b = nullptr;
  Timed(geobpe_ctx* c_, const char* n) : c(c_), name(n) {
    if (!c->prof) return;
    a = take_event(c);
    b = take_event(c);
    hipEventRecord(a, c->stream);
  }
  ~Timed() {
    if (!a) return;
    hipEventRecord(b, c->stream);
    c->pending.push_back({name, a, b});
  }
};

void collect_events(geobpe_ctx* c) {
  if (c->pending.empty()) return;
  hipStreamSynchronize(c->stream);
  for (auto& p : c->pending) {
    float ms = 0;
    hipEventElapsedTime(&ms, p.a, p.b);
    auto& t = c->ktime[p.name];
    t.first += ms;
    t.second += 1;
    c->evpool.push_back(p.a);
    c->evpool.push_back(p.b);
  }
  c->pending.clear();
}

int check_device_error(geobpe_ctx* c) {
  if (c->h_state->err_code == 0) return 0;
  const int64_t code = c->h_state->err_code, pos = c->h_state->err_pos;
  switch (code) {
    case GEOBPE_EVALUE:
      return fail(c, GEOBPE_EVALUE, "value at residue %lld does not fall into any bin", (long long)pos);
    case GEOBPE_ECAPACITY:
      return fail(c, GEOBPE_ECAPACITY, "device table capacity exceeded (site %lld)", (long long)pos);
    case GEOBPE_EHASH:
      return fail(c, GEOBPE_EHASH, "content hash collision detected (item %lld)", (long long)pos);
    default:
      return fail(c, (int)code, "device error %lld at %lld", (long long)code, (long long)pos);
  }
}

int sync_state(geobpe_ctx* c) {
  HIPCHK(c, hipMemcpyAsync(c->h_state, c->D.st, sizeof(State), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return check_device_error(c);
}

int reset_iter(geobpe_ctx* c) {
  HIPCHK(c, hipMemsetAsync((char*)c->D.st + STATE_ITER_OFF, 0, sizeof(State) - STATE_ITER_OFF, c->stream));
  return 0;
}

int alloc_keys(geobpe_ctx* c) {
  if (c->keys_ready) return 0;
  Dev& D = c->D;
  const int64_t base = c->distributed && c->global_residues > c->R ? c->global_residues : c->R;
  D.UC = 3 * base + 65536;
  int64_t hc = 1 << 16;
  while (hc < 2 * D.UC) hc <<= 1;
  D.HC = hc;
  int sh = 0;
  while ((1LL << sh) < hc) sh++;
  D.ht_shift = 64 - sh;
  int rc;
  if ((rc = dalloc(c, &D.ht_key, D.HC)) || (rc = dalloc(c, &D.ht_dense, D.HC)) || (rc = dalloc(c, &D.kh1, D.UC)) ||
      (rc = dalloc(c, &D.kh2, D.UC)) || (rc = dalloc(c, &D.klen, D.UC)) || (rc = dalloc(c, &D.krep, 3 * D.UC)) ||
      (rc = dalloc(c, &D.count, D.UC)) || (rc = dalloc(c, &D.scratch, D.UC)))
    return rc;
  if (c->distributed) {
    if ((rc = dalloc(c, &D.dcount, D.UC)) || (rc = dalloc(c, &D.touch, D.UC)) || (rc = dalloc(c, &D.touched, D.UC)))
      return rc;
    HIPCHK(c, hipMemsetAsync(D.dcount, 0, D.UC * 4, c->stream));
    HIPCHK(c, hipMemsetAsync(D.touch, 0xFF, D.UC * 4, c->stream));
  }
  D.npcap = c->R + 65536;
  D.Lcap = c->R / 2 + 1024;
  D.candcap = 1 << 20;
  if ((rc = dalloc(c, &D.np, D.npcap)) || (rc = dalloc(c, &D.ns, D.npcap)) || (rc = dalloc(c, &D.L, D.Lcap)) ||
      (rc = dalloc(c, &D.cand, D.candcap)))
    return rc;
  HIPCHK(c, hipHostMalloc((void**)&c->h_cand, sizeof(Cand) * D.candcap, hipHostMallocDefault));
  HIPCHK(c, hipMemsetAsync(D.ht_key, 0, D.HC * 8, c->stream));
  HIPCHK(c, hipMemsetAsync(D.ht_dense, 0xFF, D.HC * 4, c->stream));
  c->keys_ready = true;
  return 0;
}

// host-side content of a candidate pair: content(idL) + [g] + content(idR)
void cand_content(const geobpe_ctx* c, const Cand& k, std::vector<int32_t>& out) {
  const auto& a = c->vocab[k.idL];
  const auto& b = c->vocab[k.idR];
  out.clear();
  out.insert(out.end(), a.begin(), a.end());
  out.push_back(k.g);
  out.insert(out.end(), b.begin(), b.end());
}

// the reference priority: max count, then the smallest key string
int resolve_tie(geobpe_ctx* c, int64_t n, int32_t* W, int32_t* idL, int32_t* g, int32_t* idR) {
  if (n <= 0) return fail(c, GEOBPE_EARG, "no candidates");
  if (n > c->D.candcap) return fail(c, GEOBPE_ECAPACITY, "too many tied candidates (%lld)", (long long)n);
  int64_t best = 0;
  if (n > 1) {
    const size_t PREF = 112;
    std::vector<int32_t> buf;
    std::vector<std::string> pre((size_t)n);
    for (int64_t i = 0; i < n; i++) {
      cand_content(c, c->h_cand[i], buf);
      geobpe::render_key(buf.data(), (int64_t)buf.size(), c->B, pre[i], PREF);
      if (pre[i].size() > PREF) pre[i].resize(PREF);
    }
    std::vector<int64_t> tied;
    for (int64_t i = 0; i < n; i++) {
      if (tied.empty() || pre[i] < pre[tied[0]]) {
        tied.assign(1, i);
      } else if (pre[i] == pre[tied[0]]) {
        tied.push_back(i);
      }
    }
    best = tied[0];
    if (tied.size() > 1) {
      std::string bs, s;
      cand_content(c, c->h_cand[best], buf);
      geobpe::render_key(buf.data(), (int64_t)buf.size(), c->B, bs);
      for (size_t q = 1; q < tied.size(); q++) {
        cand_content(c, c->h_cand[tied[q]], buf);
        geobpe::render_key(buf.data(), (int64_t)buf.size(), c->B, s);
        if (s < bs) {
          bs = s;
          best = tied[q];
        }
      }
    }
  }
  const Cand& k = c->h_cand[best];
  *W = k.d;
  *idL = k.idL;
  *g = k.g;
  *idR = k.idR;
  return 0;
}

}  // namespace

// ---------------------------------------------------------------------- C ABI
extern "C" {

int geobpe_create(geobpe_ctx** out, int device, void* stream, int64_t max_vocab) {
  if (!out) return GEOBPE_EARG;
  geobpe_ctx* c = new geobpe_ctx();
  *out = c;
  c->device = device;
  c->max_vocab = max_vocab > 0 ? max_vocab : (1 << 20);
  HIPCHK(c, hipSetDevice(device));
  if (stream) {
    c->stream = (hipStream_t)stream;
  } else {
    HIPCHK(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    c->own_stream = true;
  }
  HIPCHK(c, hipHostMalloc((void**)&c->h_state, sizeof(State), hipHostMallocDefault));
  memset(c->h_state, 0, sizeof(State));
  int rc;
  if ((rc = dalloc(c, &c->D.st, 1))) return rc;
  HIPCHK(c, hipMemsetAsync(c->D.st, 0, sizeof(State), c->stream));
  int ncu = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    ncu = prop.multiProcessorCount;
  c->grid = ncu * 8;
  return 0;
}

void geobpe_destroy(geobpe_ctx* c) {
  if (!c) return;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  for (int i = 0; i < c->nallocs; i++) hipFree(c->allocs[i]);
  for (int i = 0; i < 9; i++)
    if (c->d_cols[i]) hipFree(c->d_cols[i]);
  if (c->h_state) hipHostFree(c->h_state);
  if (c->h_cand) hipHostFree(c->h_cand);
  for (auto e : c->evall) hipEventDestroy(e);
  if (c->own_stream) hipStreamDestroy(c->stream);
  delete c;
}

const char* geobpe_last_error(geobpe_ctx* c) { return c ? c->err.c_str() : "null context"; }

int geobpe_load_angles(geobpe_ctx* c, int64_t n_rows, const int64_t* h_row_off, const double* const* h_cols) {
  if (!c || n_rows < 0 || !h_row_off || !h_cols) return GEOBPE_EARG;
  if (c->R) return fail(c, GEOBPE_EARG, "corpus already loaded");
  HIPCHK(c, hipSetDevice(c->device));
  c->nrows = n_rows;
  c->row_off.assign(h_row_off, h_row_off + n_rows + 1);
  if (c->row_off[0] != 0) return fail(c, GEOBPE_EARG, "row_off[0] must be 0");
  for (int64_t r = 0; r < n_rows; r++) {
    const int64_t n = c->row_off[r + 1] - c->row_off[r];
    if (n < 1) return fail(c, GEOBPE_EARG, "row %lld is empty", (long long)r);
    c->Lmax = std::max(c->Lmax, n);
  }
  c->R = c->row_off[n_rows];
  if (c->R >= INT32_MAX / 2) return fail(c, GEOBPE_EARG, "too many residues for int32 indexing");
  Dev& D = c->D;
  D.R = c->R;
  D.nrows = n_rows;
  int rc;
  const int64_t Rp = c->R + 8;  // int4 padding for the pk scan
  if ((rc = dalloc(c, &c->d_row_off, n_rows + 1)) || (rc = dalloc(c, &D.rsym, Rp)) || (rc = dalloc(c, &D.gsym, Rp)) ||
      (rc = dalloc(c, &D.tid, Rp)) || (rc = dalloc(c, &D.tlen, Rp)) || (rc = dalloc(c, &D.tprev, Rp)) ||
      (rc = dalloc(c, &D.pk, Rp)) || (rc = dalloc(c, &D.role, Rp)))
    return rc;
  D.row_off = c->d_row_off;
  HIPCHK(c, hipMemcpyAsync(c->d_row_off, h_row_off, (n_rows + 1) * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemsetAsync(D.pk, 0xFF, Rp * 4, c->stream));
  HIPCHK(c, hipMemsetAsync(D.tid, 0xFF, Rp * 4, c->stream));
  HIPCHK(c, hipMemsetAsync(D.role, 0, Rp * 4, c->stream));
  const int need[6] = {GEOBPE_COL_PHI, GEOBPE_COL_PSI, GEOBPE_COL_OMEGA, GEOBPE_COL_TAU, GEOBPE_COL_CAC1N,
                       GEOBPE_COL_C1NCA};
  for (int q = 0; q < 6; q++) {
    const int k = need[q];
    if (!h_cols[k]) return fail(c, GEOBPE_EARG, "missing angle column %d", k);
    HIPCHK(c, hipMalloc(&c->d_cols[k], c->R * 8 + 8));
    HIPCHK(c, hipMemcpyAsync(c->d_cols[k], h_cols[k], c->R * 8, hipMemcpyHostToDevice, c->stream));
  }
  // hash powers
  const int64_t pwn = 2 * c->Lmax + 8;
  std::vector<u64> p1(pwn), p2(pwn);
  p1[0] = p2[0] = 1;
  for (int64_t i = 1; i < pwn; i++) {
    p1[i] = mulmod61(p1[i - 1], HP1);
    p2[i] = mulmod61(p2[i - 1], HP2);
  }
  u64 *dp1, *dp2;
  if ((rc = dalloc(c, &dp1, pwn)) || (rc = dalloc(c, &dp2, pwn))) return rc;
  HIPCHK(c, hipMemcpy(dp1, p1.data(), pwn * 8, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(dp2, p2.data(), pwn * 8, hipMemcpyHostToDevice));
  D.pw1 = dp1;
  D.pw2 = dp2;
  D.pwn = pwn;
  D.KC = c->max_vocab;
  if ((rc = dalloc(c, &D.vh1, D.KC)) || (rc = dalloc(c, &D.vh2, D.KC)) || (rc = dalloc(c, &D.vlen, D.KC))) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

int geobpe_angle_range(geobpe_ctx* c, double* h_minmax, int64_t* h_count) {
  if (!c || !c->R || !c->d_cols[GEOBPE_COL_TAU]) return GEOBPE_EARG;
  HIPCHK(c, hipSetDevice(c->device));
  const int nb = 512;
  double* part;
  HIPCHK(c, hipMalloc(&part, sizeof(double) * 3 * nb * GEOBPE_NTYPES));
  Cols cols;
  for (int i = 0; i < 9; i++) cols.c[i] = c->d_cols[i];
  hipLaunchKernelGGL(k_range, dim3(nb, GEOBPE_NTYPES), dim3(BLOCK), 0, c->stream, cols, c->R, part);
  std::vector<double> h(3 * nb * GEOBPE_NTYPES);
  HIPCHK(c, hipMemcpyAsync(h.data(), part, h.size() * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  hipFree(part);
  for (int t = 0; t < GEOBPE_NTYPES; t++) {
    double mn = INFINITY, mx = -INFINITY;
    int64_t cnt = 0;
    for (int b = 0; b < nb; b++) {
      const double* p = &h[((size_t)t * nb + b) * 3];
      mn = std::fmin(mn, p[0]);
      mx = std::fmax(mx, p[1]);
      cnt += (int64_t)p[2];
    }
    h_minmax[2 * t] = mn;
    h_minmax[2 * t + 1] = mx;
    if (h_count) h_count[t] = cnt;
  }
  return 0;
}

int geobpe_quantize(geobpe_ctx* c, int32_t B, const double* h_edges, double init_tau) {
  if (!c || !c->R || B < 1 || !h_edges) return GEOBPE_EARG;
  if ((int64_t)B * B * B + B >= INT32_MAX) return fail(c, GEOBPE_EARG, "too many bins (%d)", B);
  HIPCHK(c, hipSetDevice(c->device));
  c->B = B;
  Dev& D = c->D;
  D.B = B;
  D.B2 = B * B;
  D.B3 = B * B * B;
  double* de;
  HIPCHK(c, hipMalloc(&de, sizeof(double) * GEOBPE_NTYPES * (B + 1)));
  HIPCHK(c, hipMemcpyAsync(de, h_edges, sizeof(double) * GEOBPE_NTYPES * (B + 1), hipMemcpyHostToDevice, c->stream));
  Cols cols;
  for (int i = 0; i < 9; i++) cols.c[i] = c->d_cols[i];
  const int nb = (int)std::min<int64_t>(c->nrows, 65536);
  hipLaunchKernelGGL(k_quantize, dim3(std::max(nb, 1)), dim3(64), 0, c->stream, D, cols, (const double*)de, init_tau);
  HIPCHK(c, hipGetLastError());
  int rc = sync_state(c);
  hipFree(de);
  if (rc) return rc;
  for (int i = 0; i < 9; i++)
    if (c->d_cols[i]) {
      hipFree(c->d_cols[i]);
      c->d_cols[i] = nullptr;
    }
  return 0;
}

int geobpe_symbol_first(geobpe_ctx* c, int64_t row_base, int64_t* h_first) {
  if (!c || !c->B || !h_first) return GEOBPE_EARG;
  HIPCHK(c, hipSetDevice(c->device));
  const int32_t S = c->D.B3 + c->B;
  u64* df;
  HIPCHK(c, hipMalloc(&df, (size_t)S * 8));
  HIPCHK(c, hipMemsetAsync(df, 0xFF, (size_t)S * 8, c->stream));
  const int use_lds = S <= 8192;
  const int nb = (int)std::min<int64_t>((c->R + BLOCK - 1) / BLOCK, c->grid);
  hipLaunchKernelGGL(k_first, dim3(std::max(nb, 1)), dim3(BLOCK), use_lds ? S * 8 : 0, c->stream, c->D, row_base, df,
                     S, use_lds);
  HIPCHK(c, hipGetLastError());
  std::vector<u64> h(S);
  HIPCHK(c, hipMemcpyAsync(h.data(), df, (size_t)S * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  hipFree(df);
  for (int32_t s = 0; s < S; s++) h_first[s] = h[s] == ~0ULL ? INT64_MAX : (int64_t)h[s];
  return 0;
}

int geobpe_init_tokens(geobpe_ctx* c, const int32_t* h_label_of_sym, int32_t K0) {
  if (!c || !c->B || !h_label_of_sym || K0 < 0) return GEOBPE_EARG;
  if (K0 >= c->max_vocab) return fail(c, GEOBPE_ECAPACITY, "K0=%d exceeds max_vocab", K0);
  HIPCHK(c, hipSetDevice(c->device));
  const int32_t S = c->D.B3 + c->B;
  // host vocab: content of label v = its residue symbol
  c->vocab.assign(K0, {});
  std::vector<u64> vh(K0);
  std::vector<int32_t> vl(K0, 1);
  std::vector<int> seen(K0, 0);
  for (int32_t s = 0; s < S; s++) {
    const int32_t v = h_label_of_sym[s];
    if (v < 0) continue;
    if (v >= K0) return fail(c, GEOBPE_EARG, "label %d >= K0", v);
    c->vocab[v] = {s};
    vh[v] = (u64)(s + 1) % M61;
    seen[v] = 1;
  }
  for (int32_t v = 0; v < K0; v++)
    if (!seen[v]) return fail(c, GEOBPE_EARG, "label %d has no symbol", v);
  c->K0 = K0;
  int32_t* dl;
  HIPCHK(c, hipMalloc(&dl, (size_t)S * 4));
  HIPCHK(c, hipMemcpyAsync(dl, h_label_of_sym, (size_t)S * 4, hipMemcpyHostToDevice, c->stream));
  if (K0) {
    HIPCHK(c, hipMemcpyAsync(c->D.vh1, vh.data(), K0 * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->D.vh2, vh.data(), K0 * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->D.vlen, vl.data(), K0 * 4, hipMemcpyHostToDevice, c->stream));
  }
  const int nb = (int)std::min<int64_t>(c->nrows, 65536);
  hipLaunchKernelGGL(k_init_tokens, dim3(std::max(nb, 1)), dim3(64), 0, c->stream, c->D, (const int32_t*)dl);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  hipFree(dl);
  return 0;
}

int geobpe_set_distributed(geobpe_ctx* c, int on) {
  if (!c) return GEOBPE_EARG;
  if (c->keys_ready) return fail(c, GEOBPE_EARG, "set_distributed must precede bin()");
  c->distributed = on != 0;
  return 0;
}

int geobpe_set_global_residues(geobpe_ctx* c, int64_t n) {
  if (!c) return GEOBPE_EARG;
  c->global_residues = n;
  return 0;
}

static int insert_commit(geobpe_ctx* c, bool to_delta) {
  {
    Timed t(c, "assign");
    hipLaunchKernelGGL(k_assign, dim3(c->grid), dim3(BLOCK), 0, c->stream, c->D);
  }
  {
    Timed t(c, "finalize");
    hipLaunchKernelGGL(k_finalize, dim3(c->grid), dim3(BLOCK), 0, c->stream, c->D, to_delta ? 1 : 0);
  }
  HIPCHK(c, hipGetLastError());
  return 0;
}

int geobpe_bin(geobpe_ctx* c) {
  if (!c || !c->K0) return GEOBPE_EARG;
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = alloc_keys(c))) return rc;
  if ((rc = reset_iter(c))) return rc;
  {
    Timed t(c, "pair_count");
    hipLaunchKernelGGL(k_pairs_all, dim3(c->grid), dim3(BLOCK), 0, c->stream, c->D);
  }
  HIPCHK(c, hipGetLastError());
  if ((rc = insert_commit(c, c->distributed))) return rc;
  return sync_state(c);
}

int geobpe_step_select(geobpe_ctx* c, int32_t* new_id, int32_t* count) {
  if (!c || !c->keys_ready) return GEOBPE_EARG;
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = reset_iter(c))) return rc;
  {
    Timed t(c, "argmax");
    hipLaunchKernelGGL(k_argmax, dim3(c->grid), dim3(BLOCK), 0, c->stream, c->D);
    hipLaunchKernelGGL(k_cands, dim3(c->grid), dim3(BLOCK), 0, c->stream, c->D);
  }
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(c->h_state, c->D.st, sizeof(State), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if ((rc = check_device_error(c))) return rc;
  const int32_t mc = c->h_state->maxc;
  const int64_t nc = c->h_state->ncand;
  c->sel_W = -1;
  if (mc <= 0 || nc <= 0) {
    *new_id = -1;
    if (count) *count = 0;
    return 0;
  }
  const int64_t ncopy = std::min(nc, c->D.candcap);
  HIPCHK(c, hipMemcpyAsync(c->h_cand, c->D.cand, ncopy * sizeof(Cand), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  int32_t W, idL, g, idR;
  if ((rc = resolve_tie(c, nc, &W, &idL, &g, &idR))) return rc;
  const int32_t nid = (int32_t)c->vocab.size();
  if (nid >= c->max_vocab) return fail(c, GEOBPE_ECAPACITY, "vocab capacity %lld reached", (long long)c->max_vocab);
  std::vector<int32_t> content;
  Cand k{W, idL, g, idR};
  cand_content(c, k, content);
  c->vocab.push_back(std::move(content));
  c->sel_W = W;
  c->sel_new = nid;
  c->sel_count = mc;
  *new_id = nid;
  if (count) *count = mc;
  return 0;
}

int geobpe_step_apply(geobpe_ctx* c, int64_t* n_merged) {
  if (!c || c->sel_W < 0) return fail(c, GEOBPE_EARG, "step_apply without a selection");
  HIPCHK(c, hipSetDevice(c->device));
  c->tag++;
  const int32_t W = c->sel_W, nid = c->sel_new, tag = c->tag;
  const int64_t n4 = (c->R + 3) / 4;
  const int nbm = (int)std::min<int64_t>((n4 + BLOCK - 1) / BLOCK, c->grid);
  {
    Timed t(c, "mark");
    hipLaunchKernelGGL(k_mark, dim3(std::max(nbm, 1)), dim3(BLOCK), 0, c->stream, c->D, W, tag);
  }
  {
    Timed t(c, "apply");
    hipLaunchKernelGGL(k_apply, dim3(c->grid), dim3(BLOCK), 0, c->stream, c->D, W, nid, tag, c->distributed ? 1 : 0);
  }
  HIPCHK(c, hipGetLastError());
  int rc;
  if ((rc = insert_commit(c, c->distributed))) return rc;
  c->sel_W = -1;
  if (n_merged) {
    if ((rc = sync_state(c))) return rc;
    *n_merged = c->h_state->nL;
  }
  return 0;
}

int geobpe_step(geobpe_ctx* c, int32_t* new_id, int32_t* count, int64_t* n_merged) {
  if (!c || !new_id) return GEOBPE_EARG;
  if (c->distributed) return fail(c, GEOBPE_EARG, "geobpe_step in distributed mode: use step_select/apply + deltas");
  int rc;
  if ((rc = geobpe_step_select(c, new_id, count))) return rc;
  if (*new_id < 0) {
    if (n_merged) *n_merged = 0;
    return 0;
  }
  return geobpe_step_apply(c, n_merged);
}

int geobpe_delta_export(geobpe_ctx* c, void* d_out, int64_t cap, int64_t* n_records) {
  if (!c || !c->distributed || !n_records) return GEOBPE_EARG;
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = sync_state(c))) return rc;
  const int64_t n = c->h_state->ntouched;
  *n_records = n;
  if (n > cap) return fail(c, GEOBPE_ECAPACITY, "delta export needs %lld records (cap %lld)", (long long)n,
                           (long long)cap);
  hipLaunchKernelGGL(k_export, dim3(c->grid), dim3(BLOCK), 0, c->stream, c->D, (DeltaRec*)d_out, cap);
  HIPCHK(c, hipGetLastError());
  // new epoch: every key may be touched again
  const int64_t ep = c->h_state->epoch + 1;
  HIPCHK(c, hipMemcpyAsync(&c->D.st->epoch, &ep, 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemsetAsync(&c->D.st->ntouched, 0, 8, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

int geobpe_delta_import(geobpe_ctx* c, const void* d_in, int64_t n_records) {
  if (!c || !c->distributed) return GEOBPE_EARG;
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  for (int64_t off = 0; off < n_records; off += c->D.npcap) {
    const int64_t n = std::min(c->D.npcap, n_records - off);
    HIPCHK(c, hipMemsetAsync(&c->D.st->nnew_pairs, 0, 16, c->stream));  // nnew_pairs, nnew_slots
    hipLaunchKernelGGL(k_import, dim3(c->grid), dim3(BLOCK), 0, c->stream, c->D, (const DeltaRec*)d_in + off, n);
    HIPCHK(c, hipGetLastError());
    if ((rc = insert_commit(c, false))) return rc;
  }
  return sync_state(c);
}

int64_t geobpe_token_json(geobpe_ctx* c, int32_t v, char* buf, int64_t cap) {
  if (!c || v < 0 || v >= (int32_t)c->vocab.size()) return -1;
  std::string s;
  geobpe::render_key(c->vocab[v].data(), (int64_t)c->vocab[v].size(), c->B, s);
  if (buf && cap > 0) {
    const int64_t m = std::min<int64_t>((int64_t)s.size(), cap - 1);
    memcpy(buf, s.data(), m);
    buf[m] = 0;
  }
  return (int64_t)s.size();
}

int64_t geobpe_token_content(geobpe_ctx* c, int32_t v, int32_t* h_out, int64_t cap) {
  if (!c || v < 0 || v >= (int32_t)c->vocab.size()) return -1;
  const auto& x = c->vocab[v];
  if (h_out) memcpy(h_out, x.data(), sizeof(int32_t) * std::min<int64_t>(cap, (int64_t)x.size()));
  return (int64_t)x.size();
}

int64_t geobpe_vocab_count(geobpe_ctx* c) { return c ? (int64_t)c->vocab.size() : -1; }

int64_t geobpe_num_keys(geobpe_ctx* c) {
  if (!c || !c->keys_ready) return 0;
  if (sync_state(c)) return -1;
  return c->h_state->U;
}

static int row_token_offsets(geobpe_ctx* c, std::vector<int64_t>& off, int64_t** d_off) {
  int64_t* dn;
  HIPCHK(c, hipMalloc(&dn, (c->nrows + 1) * 8));
  hipLaunchKernelGGL(k_row_ntok, dim3(c->grid), dim3(BLOCK), 0, c->stream, c->D, dn);
  std::vector<int64_t> n(c->nrows);
  HIPCHK(c, hipMemcpyAsync(n.data(), dn, c->nrows * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  off.assign(c->nrows + 1, 0);
  for (int64_t r = 0; r < c->nrows; r++) off[r + 1] = off[r] + n[r];
  HIPCHK(c, hipMemcpyAsync(dn, off.data(), (c->nrows + 1) * 8, hipMemcpyHostToDevice, c->stream));
  *d_off = dn;
  return 0;
}

int64_t geobpe_num_tokens(geobpe_ctx* c) {
  if (!c || !c->R) return -1;
  std::vector<int64_t> off;
  int64_t* d;
  if (row_token_offsets(c, off, &d)) return -1;
  hipStreamSynchronize(c->stream);
  hipFree(d);
  return off.back();
}

int64_t geobpe_segmentation(geobpe_ctx* c, int32_t* h_start, int32_t* h_id, int64_t* h_row_tok_off) {
  if (!c || !c->R) return -1;
  hipSetDevice(c->device);
  std::vector<int64_t> off;
  int64_t* d_off;
  if (row_token_offsets(c, off, &d_off)) return -1;
  const int64_t T = off.back();
  if (h_row_tok_off) memcpy(h_row_tok_off, off.data(), (c->nrows + 1) * 8);
  if (h_start || h_id) {
    int32_t *ds, *di;
    if (hipMalloc(&ds, T * 4 + 4) != hipSuccess || hipMalloc(&di, T * 4 + 4) != hipSuccess) return -1;
    hipLaunchKernelGGL(k_row_seg, dim3(c->grid), dim3(BLOCK), 0, c->stream, c->D, (const int64_t*)d_off, ds, di);
    if (h_start) hipMemcpyAsync(h_start, ds, T * 4, hipMemcpyDeviceToHost, c->stream);
    if (h_id) hipMemcpyAsync(h_id, di, T * 4, hipMemcpyDeviceToHost, c->stream);
    hipStreamSynchronize(c->stream);
    hipFree(ds);
    hipFree(di);
  }
  hipStreamSynchronize(c->stream);
  hipFree(d_off);
  return T;
}

int64_t geobpe_encode(geobpe_ctx* c, int32_t* h_ids, int64_t* h_row_id_off) {
  if (!c || !c->R) return -1;
  hipSetDevice(c->device);
  std::vector<int64_t> off;
  int64_t* d_off;
  if (row_token_offsets(c, off, &d_off)) return -1;
  std::vector<int64_t> ioff(c->nrows + 1, 0);
  for (int64_t r = 0; r < c->nrows; r++) ioff[r + 1] = ioff[r] + 4 * (off[r + 1] - off[r]) - 3;
  const int64_t T = ioff.back();
  if (h_row_id_off) memcpy(h_row_id_off, ioff.data(), (c->nrows + 1) * 8);
  if (h_ids) {
    int32_t* di;
    if (hipMalloc(&di, T * 4 + 4) != hipSuccess) return -1;
    hipMemcpyAsync(d_off, ioff.data(), (c->nrows + 1) * 8, hipMemcpyHostToDevice, c->stream);
    hipLaunchKernelGGL(k_row_encode, dim3(c->grid), dim3(BLOCK), 0, c->stream, c->D, (const int64_t*)d_off, di,
                       (int32_t)c->vocab.size());
    hipMemcpyAsync(h_ids, di, T * 4, hipMemcpyDeviceToHost, c->stream);
    hipStreamSynchronize(c->stream);
    hipFree(di);
  }
  hipStreamSynchronize(c->stream);
  hipFree(d_off);
  return T;
}

int64_t geobpe_verify_counts(geobpe_ctx* c) {
  if (!c || !c->keys_ready || c->distributed) return -1;
  hipSetDevice(c->device);
  if (sync_state(c)) return -1;
  const int64_t U = c->h_state->U;
  hipMemsetAsync(c->D.scratch, 0, U * 4 + 4, c->stream);
  hipMemsetAsync(&c->D.st->nmismatch, 0, 8, c->stream);
  {
    Timed t(c, "recount");
    hipLaunchKernelGGL(k_recount, dim3(c->grid), dim3(BLOCK), 0, c->stream, c->D);
  }
  hipLaunchKernelGGL(k_compare, dim3(c->grid), dim3(BLOCK), 0, c->stream, c->D);
  if (sync_state(c)) return -1;
  return c->h_state->nmismatch;
}

int geobpe_set_profiling(geobpe_ctx* c, int on) {
  if (!c) return GEOBPE_EARG;
  collect_events(c);
  c->prof = on != 0;
  c->ktime.clear();
  return 0;
}

double geobpe_kernel_ms(geobpe_ctx* c, const char* name, int64_t* launches) {
  if (!c || !name) return -1;
  collect_events(c);
  auto it = c->ktime.find(name);
  if (it == c->ktime.end()) {
    if (launches) *launches = 0;
    return 0.0;
  }
  if (launches) *launches = it->second.second;
  return it->second.first;
}

int geobpe_synchronize(geobpe_ctx* c) {
  if (!c) return GEOBPE_EARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return check_device_error(c);
}

}  // extern "C"
