// kernels.h -- the HIP kernels of the GeoBPE engine (gfx950).  Included once, by
// geobpe.hip.  Reference behaviour cited per kernel; layout in DESIGN.md §3.
#pragma once
#include "device.h"

namespace gb {

// profiling window bracket (geobpe_marker): does nothing
__global__ void k_window_mark(int32_t tag, State* st) {
  if (tag == INT32_MIN && threadIdx.x == 64) st->nskip = 0;  // never taken; keeps the kernel non-empty
}

// timing aid (geobpe_set_hold): one thread spins for `ticks` of the 100 MHz wall clock, so
// the host can queue the launches behind it and event-timed kernels start from a backlog
// instead of waiting on the host's enqueue
__global__ void k_hold(int64_t ticks) {
  const int64_t t0 = (int64_t)wall_clock64();
  while ((int64_t)wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

// ====================================================================== prologue
__constant__ int32_t c_type_col[GEOBPE_NTYPES] = {GEOBPE_COL_TAU, GEOBPE_COL_CAC1N, GEOBPE_COL_C1NCA,
                                                  GEOBPE_COL_PSI, GEOBPE_COL_OMEGA, GEOBPE_COL_PHI};
struct Cols {
  const double* c[9];
};

// per (workgroup, type) min / max / count of the wrapped non-NaN non-zero values
// (the inputs of np.histogram in BPE._init_thresholds, bpe.py:840-850)
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

// residue / junction symbols: SURVEY.md App. A with the Tokenizer index maps
// (tokenizer.py:131-167) and get_ind (bpe.py:1164-1189)
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

// after the bin pass: the merge loop's token records, whole ({label, 1 | 16-bit junction
// symbol << 16, previous slot, pair key}: one 16-B store per residue, consecutive lanes on
// consecutive records), and the 16-bit junction symbols.  Round 4's k_pack stored pk and the
// length word into the records' 2nd and 4th words, 4-B stores at a 16-B lane stride, ~285 us
// at C3.  (Every token is one residue here; g starts its chain iff gsym[g - 1] < 0.)  Measured
// and dropped: reading the listed pairs' keys here instead of a fix-up kernel, four
// residues per thread, 2-8 residues per thread in flight.
__global__ __launch_bounds__(BLOCK) void k_pack(Dev D) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < D.R; g += (int64_t)gridDim.x * blockDim.x) {
    const int32_t lab = D.lab0[g], gs = D.gsym[g], k = D.pk[g];
    const int32_t gp = g > 0 ? D.gsym[g - 1] : -1;  // (the previous lane's line: a cache hit)
    const uint32_t g16 = gs < 0 ? 0xFFFFu : (uint32_t)gs;
    D.tok[g] = make_int4(lab, D.gs16 ? (int32_t)(1u | (g16 << 16)) : 1, gp >= 0 ? (int32_t)(g - 1) : -1, k);
    if (D.gs16) D.gs16[g] = (uint16_t)g16;
  }
}

__global__ __launch_bounds__(64) void k_init_tokens(Dev D, const int32_t* label_of_sym) {
  for (int64_t r = blockIdx.x; r < D.nrows; r += gridDim.x) {
    const int64_t a = D.row_off[r], b = D.row_off[r + 1];
    for (int64_t g = a + threadIdx.x; g < b; g += blockDim.x) {
      const int32_t sy = D.rsym[g];
      const int32_t lab = label_of_sym[sy];
      D.tok[g] = make_int4(lab, 1, (g == a) ? -1 : (int32_t)(g - 1), 0);
      D.lab0[g] = lab;
      D.pk[g] = -1;
    }
  }
}

// ====================================================================== region emitters
// new pair into this workgroup's region (LDS cursor), spilling to the overflow list
__device__ inline void emit_pair(const Dev& D, int32_t* s_cnt, int32_t target, int32_t slot, int32_t len,
                                 int32_t delta, u64 h1, u64 h2) {
  NewPair e;
  e.target = target;
  e.slot = slot;
  e.len = len;
  e.delta = delta;
  e.h1 = h1;
  e.h2 = h2;
  const int32_t j = atomicAdd(s_cnt, 1);
  if (j < D.RC) {
    D.np[(int64_t)blockIdx.x * D.RC + j] = e;
  } else {
    const int64_t k = atomicAdd((unsigned long long*)&D.st->np_ovf, 1ULL);
    if (k < D.ovf_cap)
      D.npovf[k] = e;
    else
      set_error(D, GEOBPE_ECAPACITY, -3);
  }
}

// A pair key is named by its key-table slot (the key id): the thread whose CAS
// claims the slot writes the key's payload there at once and lists the slot in
// klist; a finder has the id as soon as its probe matches -- nothing to wait for.
__device__ inline void claim_payload(const Dev& D, int32_t slot, u64 h1, u64 h2, int32_t len, int32_t idL, int32_t g,
                                     int32_t idR) {
  D.kh1[slot] = h1;
  D.kh2[slot] = h2;
  D.klen[slot] = len;
  D.krep[3 * (int64_t)slot + 0] = idL;
  D.krep[3 * (int64_t)slot + 1] = g;
  D.krep[3 * (int64_t)slot + 2] = idR;
}

__device__ inline void klist_put(const Dev& D, int64_t k, int32_t slot) {
  if (k < D.KCAP)
    D.klist[k] = slot;
  else
    set_error(D, GEOBPE_ECAPACITY, -5);
}

// a claimed slot joins this workgroup's claim region (klist entries at region close)
__device__ inline void note_claim(const Dev& D, int32_t* s_ns, int32_t slot) {
  const int32_t j = atomicAdd(s_ns, 1);
  if (j < D.RC)
    D.ns[(int64_t)blockIdx.x * D.RC + j] = slot;
  else {  // rare: listed right away
    klist_put(D, (int64_t)atomicAdd((unsigned long long*)&D.st->U, 1ULL), slot);
  }
}

// insert (or find) a pair key and emit the pair
__device__ inline void add_pair(const Dev& D, int32_t* s_np, int32_t* s_ns, int32_t target, u64 h1, u64 h2,
                                int32_t len, int32_t idL, int32_t g, int32_t idR, int32_t delta) {
  bool claimed;
  const int32_t slot = ht_insert(D, h1, h2, len, &claimed);
  if (slot < 0) return;
  if (claimed) {
    claim_payload(D, slot, h1, h2, len, idL, g, idR);
    note_claim(D, s_ns, slot);
  }
  emit_pair(D, s_np, target, slot, len, delta, h1, h2);
}

// end of a region kernel: this workgroup's claimed keys join klist (one global
// reservation); the pair count of a bin / import region is published
__device__ inline void close_claims(const Dev& D, int32_t* s_ns) {
  __shared__ int64_t s_base;
  __syncthreads();
  const int32_t n = min(*s_ns, (int32_t)D.RC);
  if (threadIdx.x == 0) {
    s_base = n ? (int64_t)atomicAdd((unsigned long long*)&D.st->U, (unsigned long long)n) : 0;
  }
  __syncthreads();
  const int32_t* reg = D.ns + (int64_t)blockIdx.x * D.RC;
  for (int32_t i = threadIdx.x; i < n; i += blockDim.x) klist_put(D, s_base + i, reg[i]);
}
__device__ inline void close_regions(const Dev& D, int32_t* s_np, int32_t* s_ns) {
  close_claims(D, s_ns);
  if (threadIdx.x == 0) D.npcnt[blockIdx.x] = min(*s_np, (int32_t)D.RC);
}

// ====================================================================== histogram
// BPE.bin (bpe.py:1431-1474): every live adjacent pair -> content hash -> key
__global__ __launch_bounds__(ABLOCK) void k_pairs_all(Dev D) {
  __shared__ int32_t s_np, s_ns;
  if (threadIdx.x == 0) s_np = s_ns = 0;
  __syncthreads();
  const int64_t SC = (D.R + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * SC, hi = min(D.R, lo + SC);
  for (int64_t g = lo + threadIdx.x; g < hi; g += blockDim.x) {
    const int4 tg = D.tok[g];
    const int32_t L = tg.x;
    if (L < 0) continue;
    const int32_t xlen = tok_len(tg.y);
    const int32_t e = (int32_t)g + xlen - 1;
    if (D.rsym[e] >= D.B3) continue;  // last token of its chain
    const int4 te = D.tok[e + 1];
    const int32_t Rr = te.x;
    const int32_t gl = D.gsym[e];
    const int32_t ylen = tok_len(te.y);
    u64 h1, h2;
    combine(D, D.vh1[L], D.vh2[L], gl, D.vh1[Rr], D.vh2[Rr], ylen, h1, h2);
    add_pair(D, &s_np, &s_ns, (int32_t)g, h1, h2, xlen + ylen, L, gl, Rr, 1);
  }
  close_regions(D, &s_np, &s_ns);
}

#include "bin_dense.h"

// pair -> key id into pk, counts via LDS-staged partial counts (+ the hot-list
// crossing check on the global counts); the key's payload must be this content
__device__ inline void finalize_one(const Dev& D, AggBig& agg, HotApp& hot, const NewPair& e, int64_t j, bool to_delta,
                                    int32_t th) {
  const int32_t d = e.slot;
  if (!key_is(D, d, e.h1, e.h2, e.len)) {
    set_error(D, GEOBPE_EHASH, j);
    return;
  }
  if (e.target >= 0) D.pk[e.target] = d;
  agg_add_hot(agg, D, hot, d, e.delta, to_delta, th);
}

// a hot-list rebuild iteration (k_mark chose it; run by k_apply's grid):
// counter `build` (zeroed by k_mark) and clist = every key with count >= th.
// Two coalesced passes over this workgroup's share of klist; one global
// reservation per workgroup.
__device__ void rebuild_hot_list(const Dev& D, int32_t th, int32_t build, int32_t blk, int32_t nblk) {
  __shared__ int32_t s_red[ABLOCK / 64];
  __shared__ int64_t s_base;
  State* st = D.st;
  const int64_t U = min(st->U, D.KCAP);
  const int64_t per = (U + nblk - 1) / nblk;
  const int64_t lo = (int64_t)blk * per, hi = min(U, lo + per);
  constexpr int UNR = 16;  // loads in flight per thread
  int32_t n = 0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += UNR * ABLOCK) {
    int32_t d[UNR];
#pragma unroll
    for (int u = 0; u < UNR; u++) d[u] = i + u * ABLOCK < hi ? D.klist[i + u * ABLOCK] : -1;
#pragma unroll
    for (int u = 0; u < UNR; u++) n += d[u] >= 0 && D.count[d[u]] >= th;
  }
  int32_t tot;
  const int32_t ex = block_excl_scan(n, &tot, s_red);
  if (threadIdx.x == 0)
    s_base = tot ? (int64_t)atomicAdd((unsigned long long*)&st->ncl2[build], (unsigned long long)tot) : 0;
  __syncthreads();
  int64_t j = s_base + ex;
  for (int64_t i = lo + threadIdx.x; i < hi; i += UNR * ABLOCK) {
    int32_t d[UNR];
#pragma unroll
    for (int u = 0; u < UNR; u++) d[u] = i + u * ABLOCK < hi ? D.klist[i + u * ABLOCK] : -1;
#pragma unroll
    for (int u = 0; u < UNR; u++)
      if (d[u] >= 0 && D.count[d[u]] >= th) D.clist[j++] = d[u];  // j < U <= KCAP
  }
  if (blk == 0 && threadIdx.x == 0) {
    st->cl_act = build;
    st->theta = th;
    st->cl_valid = 1;
    st->cl_measured = 0;
  }
}
__device__ inline void rebuild_hot_list(const Dev& D, int32_t th, int32_t build) {
  rebuild_hot_list(D, th, build, blockIdx.x, gridDim.x);
}

// a measure iteration: the global maximum count (the hot list must be rebuilt
// from scratch and its threshold needs it)
__device__ void measure_max(const Dev& D, int32_t blk, int32_t nblk) {
  __shared__ int32_t s_red[ABLOCK / 64];
  const int64_t U = min(D.st->U, D.KCAP);
  const int64_t per = (U + nblk - 1) / nblk;
  const int64_t lo = (int64_t)blk * per, hi = min(U, lo + per);
  constexpr int UNR = 16;
  int32_t m = 0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += UNR * ABLOCK) {
    int32_t d[UNR];
#pragma unroll
    for (int u = 0; u < UNR; u++) d[u] = i + u * ABLOCK < hi ? D.klist[i + u * ABLOCK] : -1;
#pragma unroll
    for (int u = 0; u < UNR; u++)
      if (d[u] >= 0) m = max(m, D.count[d[u]]);
  }
  m = block_max(m, s_red);
  if (threadIdx.x == 0 && m > 0) atomicMax((unsigned long long*)&D.st->cl_measured, (unsigned long long)m);
}
__device__ inline void measure_max(const Dev& D) { measure_max(D, blockIdx.x, gridDim.x); }

__global__ __launch_bounds__(ABLOCK) void k_finalize(Dev D, int to_delta) {
  __shared__ AggBig agg;
  __shared__ HotApp hot;
  const int32_t th = D.st->theta;
  agg_init(agg);
  hot_init(hot);
  const int32_t n = D.npcnt[blockIdx.x];
  const NewPair* reg = D.np + (int64_t)blockIdx.x * D.RC;
  for (int32_t i = threadIdx.x; i < n; i += blockDim.x) finalize_one(D, agg, hot, reg[i], i, to_delta != 0, th);
  const int64_t novf = min(D.st->np_ovf, D.ovf_cap);
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < novf; k += (int64_t)gridDim.x * blockDim.x)
    finalize_one(D, agg, hot, D.npovf[k], k, to_delta != 0, th);
  agg_flush_hot(agg, D, hot, to_delta != 0, th);
}

#include "exchange.h"
#include "merge.h"

// ====================================================================== argmax + tie-break
// the reference key string json.dumps(geo, sort_keys=True) of a content, char by
// char (same rendering as keyjson.h::render_key)
struct JGen {
  const int32_t *A, *C;
  int32_t nA, g, nC;
  int32_t B, B2, B3, r, lam;
  int32_t sec, item, len, pos;
  char* buf;  // 24 chars of LDS per generator (private arrays would put the kernel on scratch)

  // (a select between two global pointers, then g by value: a pointer to g would
  // put the generator on the scratch stack)
  __device__ int32_t sym(int32_t k) const {
    const int32_t* p = k < nA ? A + k : C + max(k - nA - 1, 0);
    const int32_t v = *p;
    return k == nA ? g : v;
  }
  __device__ void init(const int32_t* a, int32_t na, int32_t gg, const int32_t* c, int32_t nc, int32_t b, char* lds) {
    buf = lds;
    A = a;
    nA = na;
    g = gg;
    C = c;
    nC = nc;
    B = b;
    B2 = b * b;
    B3 = B2 * b;
    const int32_t n = na + 1 + nc;
    r = (n + 1) / 2;
    lam = sym(n - 1) >= B3 ? 1 : 0;
    sec = -1;
    item = len = pos = 0;
  }
  __device__ int32_t sec_len(int32_t s) const {
    switch (s) {
      case 0: case 3: case 7: return r - lam;
      case 1: case 5: case 6: return r - 1;
      default: return r;
    }
  }
  __device__ int32_t value(int32_t s, int32_t i) const {
    switch (s) {
      case 1: return sym(2 * i + 1) / B % B;   // C:1N:1CA
      case 3: return sym(2 * i) / B % B;       // CA:C:1N
      case 5: return sym(2 * i + 1) / B2;      // omega
      case 6: return sym(2 * i + 1) % B;       // phi
      case 7: return sym(2 * i) % B;           // psi
      case 8: {                                // tau
        const int32_t x = sym(2 * i);
        return x >= B3 ? x - B3 : x / B2;
      }
      default: return 0;                       // bond lists (std_bonds)
    }
  }
  __device__ void put(const char* s) {
    while (*s) buf[len++] = *s++;
  }
  __device__ void put_int(int32_t v) {
    int n = 1;
    for (int32_t x = v; x >= 10; x /= 10) n++;
    for (int k = n - 1; k >= 0; k--) {
      buf[len + k] = (char)('0' + v % 10);
      v /= 10;
    }
    len += n;
  }
  __device__ bool refill() {
    len = pos = 0;
    if (sec == 9) return false;
    if (sec == -1) {
      put("{\"0C:1N\": [");
      sec = 0;
      item = 0;
      return true;
    }
    if (item < sec_len(sec)) {
      if (item > 0) put(", ");
      put_int(value(sec, item));
      item++;
      return true;
    }
    if (sec == 8) {
      put("]}");
      sec = 9;
      return true;
    }
    sec++;
    item = 0;
    put("], \"");
    switch (sec) {
      case 1: put("C:1N:1CA"); break;
      case 2: put("CA:C"); break;
      case 3: put("CA:C:1N"); break;
      case 4: put("N:CA"); break;
      case 5: put("omega"); break;
      case 6: put("phi"); break;
      case 7: put("psi"); break;
      default: put("tau"); break;
    }
    put("\": [");
    return true;
  }
  __device__ int next() {
    while (pos >= len)
      if (!refill()) return -1;
    return (unsigned char)buf[pos++];
  }
};

// generator over key d's reference string: content(L) ++ [g] ++ content(R)
__device__ inline void key_gen(const Dev& D, int32_t d, JGen& x, char* lds) {
  const int32_t L = D.krep[3 * d], g = D.krep[3 * d + 1], Rr = D.krep[3 * d + 2];
  const int64_t a0 = D.voff[L], a1 = D.voff[L + 1], c0 = D.voff[Rr], c1 = D.voff[Rr + 1];
  x.init(D.vsym + a0, (int32_t)(a1 - a0), g, D.vsym + c0, (int32_t)(c1 - c0), D.B, lds);
}

// true iff key a's reference string < key b's (Python str order); lds: 48 chars
// of this thread's LDS
__device__ inline bool key_less(const Dev& D, int32_t a, int32_t b, char* lds) {
  JGen x, y;
  key_gen(D, a, x, lds);
  key_gen(D, b, y, lds + 24);
  for (;;) {
    const int ca = x.next(), cb = y.next();
    if (ca != cb) return ca < cb;
    if (ca < 0) return false;
  }
}

// The same order, compared item by item by a whole wave (the char generator
// above costs ~100 instructions per character on one lane: 30-250 us for the
// long tied keys of late merges).  The key string is nine lists
// '{"0C:1N": [I0], "C:1N:1CA": [I1], ... "tau": [I8]}' with Is = ", ".join(str(v)).
// Two strings first differ inside the first list s that differs, at its first
// differing item i:
//   * one list ended at i: its ']' sorts after the other's ',' or digit -> it is larger;
//   * items x != y: decimal strings compared char-wise; when one is a prefix of
//     the other the shorter one's terminator decides (',' < digit < ']').
struct KSeq {  // content(L) ++ [g] ++ content(R)
  const int32_t *A, *C;
  int32_t nA, g, nC;
};
__device__ inline int32_t kseq_sym(const KSeq& q, int32_t k) {
  const int32_t* p = k < q.nA ? q.A + k : q.C + max(k - q.nA - 1, 0);
  const int32_t v = *p;
  return k == q.nA ? q.g : v;
}
__device__ inline int32_t ksec_len(int s, int32_t r, int32_t lam) {
  switch (s) {
    case 0: case 3: case 7: return r - lam;
    case 1: case 5: case 6: return r - 1;
    default: return r;
  }
}
__device__ inline int32_t ksec_val(const KSeq& q, int s, int32_t i, int32_t B, int32_t B2, int32_t B3) {
  switch (s) {
    case 1: return kseq_sym(q, 2 * i + 1) / B % B;  // C:1N:1CA
    case 3: return kseq_sym(q, 2 * i) / B % B;      // CA:C:1N
    case 5: return kseq_sym(q, 2 * i + 1) / B2;     // omega
    case 6: return kseq_sym(q, 2 * i + 1) % B;      // phi
    case 7: return kseq_sym(q, 2 * i) % B;          // psi
    case 8: {                                       // tau
      const int32_t x = kseq_sym(q, 2 * i);
      return x >= B3 ? x - B3 : x / B2;
    }
    default: return 0;  // bond lists (std_bonds)
  }
}
__device__ inline int ndigits(int32_t v) {
  int n = 1;
  for (; v >= 10; v /= 10) n++;
  return n;
}
// str(x) + (']' if xlast else ',') < str(y) + (']' if ylast else ',') for x != y
__device__ inline bool item_less(int32_t x, bool xlast, int32_t y, bool ylast) {
  const int dx = ndigits(x), dy = ndigits(y);
  if (dx == dy) return x < y;
  if (dx < dy) {
    int32_t yp = y;
    for (int k = dx; k < dy; k++) yp /= 10;
    return yp != x ? x < yp : !xlast;  // x a prefix of y: x's terminator against a digit
  }
  int32_t xp = x;
  for (int k = dy; k < dx; k++) xp /= 10;
  return xp != y ? xp < y : ylast;
}
// key string of a < key string of b; every lane of the wave calls it with the
// same arguments and gets the same answer
__device__ inline bool wave_key_less(const KSeq& a, const KSeq& b, int32_t B) {
  const int32_t B2 = B * B, B3 = B2 * B;
  const int lane = (int)(threadIdx.x & 63);
  const int32_t na = a.nA + 1 + a.nC, nb = b.nA + 1 + b.nC;
  const int32_t ra = (na + 1) / 2, rb = (nb + 1) / 2;
  const int32_t lama = kseq_sym(a, na - 1) >= B3 ? 1 : 0, lamb = kseq_sym(b, nb - 1) >= B3 ? 1 : 0;
  for (int s = 0; s < 9; s++) {
    const int32_t la = ksec_len(s, ra, lama), lb = ksec_len(s, rb, lamb);
    if (s == 0 || s == 2 || s == 4) {  // lists of zeros: the shorter one is larger
      if (la != lb) return la > lb;
      continue;
    }
    const int32_t m = max(la, lb);
    for (int32_t i0 = 0; i0 < m; i0 += 64) {
      const int32_t i = i0 + lane;
      const bool ia = i < la, ib = i < lb;
      int32_t va = 0, vb = 0;
      bool diff = false;
      if (ia && ib) {
        va = ksec_val(a, s, i, B, B2, B3);
        vb = ksec_val(b, s, i, B, B2, B3);
        diff = va != vb;
      } else {
        diff = ia != ib;
      }
      const unsigned long long mask = __ballot(diff);
      if (mask) {
        const int first = __ffsll((long long)mask) - 1;
        const int res = !ia ? 0 : (!ib ? 1 : (item_less(va, i == la - 1, vb, i == lb - 1) ? 1 : 0));
        return __shfl(res, first, 64) != 0;
      }
    }
  }
  return false;
}

__device__ inline KSeq key_seq(const Dev& D, int32_t d) {
  const int32_t L = D.krep[3 * (int64_t)d], g = D.krep[3 * (int64_t)d + 1], Rr = D.krep[3 * (int64_t)d + 2];
  const int64_t a0 = D.voff[L], a1 = D.voff[L + 1], c0 = D.voff[Rr], c1 = D.voff[Rr + 1];
  return KSeq{D.vsym + a0, D.vsym + c0, (int32_t)(a1 - a0), g, (int32_t)(c1 - c0)};
}

// BPE.step's argmax (bpe.py:1796-1800, SortedDict peekitem(0)): every key with
// count >= theta is in clist[0..n), so when the list maximum m >= theta it is the
// global maximum and every key tied at m is in the list.  Otherwise (or when the
// list has grown long while m >= 4 theta) the launch triple is a rebuild
// iteration with theta_new = max(1, m/2) <= the true maximum; an invalid list
// is first re-measured.  Ties: the smallest reference key string
// (bpe.py:1469-1471) via the device JSON generator.
//
// k_select: one workgroup of SBLOCK threads (16 waves).  Every thread keeps
// SEL_UNR list entries in flight (one round covers 4096 entries: the lists of a
// C3/C5 run hold <= ~5 k), so the scan is one or two rounds of dependent list -> count
// gathers.  The keys tied at the maximum are collected in LDS, their contents
// staged in LDS, and a wave-per-comparison tournament (wave_key_less) picks the
// smallest reference string.  It records the decision in Sel[par], the
// merge-log entry and the new token's hash (_tokens[n] = json.loads(key),
// bpe.py:1857-1860; its content is written by k_apply's workgroup 0).  More than
// SEL_TMAX tied keys (runs to exhaustion) fall back to the char generator.
// (Measured: the char-generator tie tree cost 30-250 us a merge for the 10-30 tied
// long keys of late merges; a 64-workgroup scan with a last-arriver reduction
// paid ~6 us of release/acquire fences and tickets for nothing at these lengths.)
constexpr int SBLOCK = 1024;
constexpr int SEL_UNR = 4;  // list entries in flight per thread (A/B: 8 is no faster)
constexpr int SEL_TMAX = SBLOCK;  // staged candidates
constexpr int SEL_SYMS = 6144;    // staged content symbols (24 KB)

// block-wide smallest reference key string among the threads' candidates (-1 = none)
__device__ inline int32_t block_min_key(const Dev& D, int32_t best, int32_t* s_best, char* jb) {
  s_best[threadIdx.x] = best;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      const int32_t a = s_best[threadIdx.x], b = s_best[threadIdx.x + o];
      if (a < 0 || (b >= 0 && b != a && key_less(D, b, a, jb))) s_best[threadIdx.x] = b;
    }
    __syncthreads();
  }
  const int32_t r = s_best[0];
  __syncthreads();
  return r;
}

struct SelStage {  // the tied keys and LDS copies of their contents
  int32_t key[SEL_TMAX];
  int32_t off[SEL_TMAX];
  int32_t idx[SEL_TMAX];
  KSeq seq[SEL_TMAX];
  int32_t sym[SEL_SYMS];
  int32_t nt;
};

// tournament over the tied keys (indices 0..nt-1 into S.seq), one wave per
// comparison; returns the index of the smallest key string
__device__ inline int32_t wave_tournament(SelStage& S, int32_t nt, int32_t B) {
  const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((int)threadIdx.x < nt) S.idx[threadIdx.x] = threadIdx.x;
  __syncthreads();
  for (int32_t cnt = nt; cnt > 1;) {
    const int32_t up = (cnt + 1) / 2;
    for (int32_t p = wave; p < cnt - up; p += nw) {
      const int32_t ia = S.idx[p], ib = S.idx[p + up];
      const bool bl = S.key[ia] != S.key[ib] && wave_key_less(S.seq[ib], S.seq[ia], B);
      if ((threadIdx.x & 63) == 0 && bl) S.idx[p] = ib;
    }
    __syncthreads();
    cnt = up;
  }
  const int32_t r = S.idx[0];
  __syncthreads();
  return r;
}

// the posting index must be rebuilt before a merge of count m: never built, a log
// append was lost, or the log pool cannot take the merge's new pairs (<= 2 per
// occurrence, <= R in all; each owner may open one more chunk)
__device__ inline bool post_stale(const Dev& D, int64_t m) {
  const State* st = D.st;
  const int64_t need = (min(2 * m, D.R) + D.CHUNK - 1) / D.CHUNK + D.NBA;
  return st->post_valid == 0 || st->plog_ovf != 0 || st->pool_used + need > D.POOL_CH;
}

// plain loads in a kernel that reads state written by earlier launches; loads that
// bypass this CU's L1 (agent scope) where the same launch changes the data with
// atomics (the persistent late-merge kernel, tail.h)
template <bool COH, class T>
__device__ inline T ldc(const T* p) {
  if constexpr (COH)
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    return *p;
}

// the argmax + tie-break of one iteration (every thread of the workgroup calls it): the
// decision goes to Sel[par] and, when lsel is given, to LDS (thread 0 writes both)
template <bool COH>
__device__ void select_core(const Dev& D, int par, SelStage& S, int32_t* s_red, Sel* lsel, int32_t run_end = 0) {
  State* st = D.st;
  Sel* out = D.sel + par;
  const bool rec = threadIdx.x == 0;
  Sel o{};
  auto publish = [&]() {
    *out = o;
    if (lsel) *lsel = o;
  };
  dbg_stamp(D, 20);  // (debug timeline slots 20-26: k_select phases)
  const int32_t act = ldc<COH>(&st->cl_act);
  // the first SEL_UNR * SBLOCK list entries are loaded with the state (clist
  // capacity KCAP >= SEL_UNR * SBLOCK; entries past n are masked below)
  int32_t d0[SEL_UNR];
#pragma unroll
  for (int q = 0; q < SEL_UNR; q++) d0[q] = D.clist[threadIdx.x + q * SBLOCK];
  const int64_t n = ldc<COH>(&st->ncl2[act]);
  const int32_t th = ldc<COH>(&st->theta), iter = ldc<COH>(&st->iter), K = ldc<COH>(&st->K);
  const bool valid = ldc<COH>(&st->cl_valid) != 0;
  if (ldc<COH>(&st->done)) {
    if (rec) {
      o.decision = SEL_DONE;
      publish();
    }
    return;
  }
  if (run_end > 0 && iter >= run_end - 1) {  // the run's merges are made: an idle iteration
    if (rec) {
      o.decision = SEL_IDLE;
      publish();
    }
    return;
  }
  if (!valid) {  // no usable list: measure the maximum, then rebuild at half of it
    if (!rec) return;
    const Sel& prev = D.sel[par ^ 1];
    const bool measured = prev.decision == SEL_SKIP && (prev.skip & SKIP_MEASURE);
    const int64_t ms = measured ? ldc<COH>(&st->cl_measured) : 0;
    if (measured && ms == 0) {
      o.decision = SEL_DONE;
      o.maxc = 0;
    } else {
      o.decision = SEL_SKIP;
      o.skip = measured ? SKIP_HOT : SKIP_MEASURE;
      o.theta_new = (int32_t)max((int64_t)1, ms / 2);
      o.build = act ^ 1;
      st->ncl2[act ^ 1] = 0;  // (no mark workgroup reads the idle counter)
    }
    publish();
    return;
  }
  // ---- pass over the list: SEL_UNR entries per thread in flight; keep this thread's maximum
  int32_t m = 0, mkey = -1, mcnt = 0;
  for (int64_t i0 = threadIdx.x; i0 < n; i0 += SEL_UNR * SBLOCK) {
    int32_t d[SEL_UNR], c[SEL_UNR];
#pragma unroll
    for (int q = 0; q < SEL_UNR; q++) {
      const int64_t i = i0 + (int64_t)q * SBLOCK;
      d[q] = i < n ? (i0 < SBLOCK ? d0[q] : D.clist[i]) : -1;
    }
#pragma unroll
    for (int q = 0; q < SEL_UNR; q++) c[q] = d[q] >= 0 ? ldc<COH>(&D.count[d[q]]) : 0;
#pragma unroll
    for (int q = 0; q < SEL_UNR; q++) {
      if (c[q] > m) {
        m = c[q];
        mkey = d[q];
        mcnt = 1;
      } else if (c[q] == m && d[q] >= 0 && c[q] > 0) {
        mcnt++;
      }
    }
  }
  if (rec) S.nt = 0;
  dbg_stamp(D, 21);
  const int32_t gm = block_max(m, s_red);
  // the payload of a key at the maximum, loaded by its thread while the ties are collected:
  // when one key holds the maximum (nt == 1, the common case) that thread publishes without
  // another round trip
  int32_t pL = 0, pg = 0, pR = 0, pwl = 0, pkn = 0, pko = 0;
  u64 pw1 = 0, pw2 = 0;
  if (mkey >= 0 && m == gm && mcnt == 1) {
    pL = D.krep[3 * (int64_t)mkey];
    pg = D.krep[3 * (int64_t)mkey + 1];
    pR = D.krep[3 * (int64_t)mkey + 2];
    pw1 = D.kh1[mkey];
    pw2 = D.kh2[mkey];
    pwl = D.klen[mkey];
    if (D.kp_n) {
      pkn = ldc<COH>(&D.kp_n[mkey]);
      pko = D.kp_off[mkey];
    }
  }
  dbg_stamp(D, 22);
  const bool hot = gm < th || (n > CL_MIN_SHRINK && (int64_t)gm >= 4 * (int64_t)th);
  if (hot && th <= 1 && gm == 0) {  // every key with count >= 1 is listed: nothing left
    if (rec) {
      o.decision = SEL_DONE;
      o.maxc = 0;
      publish();
    }
    return;
  }
  if (hot) {
    if (rec) {
      o.decision = SEL_SKIP;
      o.skip = SKIP_HOT;
      o.theta_new = max(1, gm / 2);
      o.build = act ^ 1;
      st->ncl2[act ^ 1] = 0;
      publish();
    }
    return;
  }
  if (K >= D.KC) {
    if (rec) {
      set_error(D, GEOBPE_ECAPACITY, -9);
      o.decision = SEL_DONE;
      publish();
    }
    return;
  }
  // ---- the keys tied at the maximum (a thread with several re-reads its entries;
  // a key listed twice is one candidate twice, harmless)
  if (m == gm) {
    if (mcnt == 1) {
      const int32_t j = atomicAdd(&S.nt, 1);
      if (j < SEL_TMAX) S.key[j] = mkey;
    } else {
      for (int64_t i = threadIdx.x; i < n; i += SBLOCK) {
        const int32_t d = D.clist[i];
        if (ldc<COH>(&D.count[d]) == gm) {
          const int32_t j = atomicAdd(&S.nt, 1);
          if (j < SEL_TMAX) S.key[j] = d;
        }
      }
    }
  }
  __syncthreads();
  dbg_stamp(D, 23);
  const int32_t nt = S.nt;
  const int32_t t = threadIdx.x;
  int32_t W;
  if (nt == 1) {
    W = S.key[0];
  } else if (nt <= SEL_TMAX) {
    // the candidates' contents (global), their staging offsets (one candidate per thread)
    int32_t len = 0;
    if (t < nt) {
      S.seq[t] = key_seq(D, S.key[t]);
      len = S.seq[t].nA + S.seq[t].nC;
    }
    int32_t tot;
    const int32_t o2 = block_excl_scan(len, &tot, s_red);
    if (t < nt) S.off[t] = o2;
    __syncthreads();
    if (tot <= SEL_SYMS) {  // copy into LDS, one candidate per wave, 64 symbols a step
      for (int32_t c = t >> 6; c < nt; c += SBLOCK / 64) {
        const KSeq q = S.seq[c];
        int32_t* dst = S.sym + S.off[c];
        for (int32_t k = t & 63; k < q.nA; k += 64) dst[k] = q.A[k];
        for (int32_t k = t & 63; k < q.nC; k += 64) dst[q.nA + k] = q.C[k];
      }
      __syncthreads();
      if (t < nt) {
        S.seq[t].A = S.sym + S.off[t];
        S.seq[t].C = S.sym + S.off[t] + S.seq[t].nA;
      }
      __syncthreads();
    }  // else: the tournament compares in global memory
    dbg_stamp(D, 24);
    W = S.key[wave_tournament(S, nt, D.B)];
    dbg_stamp(D, 25);
  } else {
    // more tied keys than the staging holds (runs to exhaustion): the char
    // generator over the list, 256 threads (48 chars of LDS each, in S.sym)
    char* jb = (char*)S.sym + 48 * (t & 255);
    int32_t best = -1;
    if (t < 256)
      for (int64_t i = t; i < n; i += 256) {
        const int32_t d = D.clist[i];
        if (ldc<COH>(&D.count[d]) == gm && (best < 0 || (d != best && key_less(D, d, best, jb)))) best = d;
      }
    W = block_min_key(D, best, S.idx, jb);
  }
  const bool solo = nt == 1;  // (then exactly one thread has m == gm with mcnt == 1: it listed W)
  if (solo ? (m == gm && mcnt == 1) : rec) {
    const int32_t L = solo ? pL : D.krep[3 * (int64_t)W], g = solo ? pg : D.krep[3 * (int64_t)W + 1],
                  Rr = solo ? pR : D.krep[3 * (int64_t)W + 2];
    const u64 w1 = solo ? pw1 : D.kh1[W], w2 = solo ? pw2 : D.kh2[W];
    const int32_t wl = solo ? pwl : D.klen[W];
    D.vh1[K] = w1;
    D.vh2[K] = w2;
    D.vlen[K] = wl;
    LogRec lr;
    lr.nid = K;
    lr.count = gm;
    lr.W = W;
    lr.idL = L;
    lr.g = g;
    lr.idR = Rr;
    lr.nmerged = 0;
    D.log[iter] = lr;
    o.decision = SEL_MERGE;
    o.skip = 0;
    o.rebuild = post_stale(D, gm) ? 1 : 0;
    o.wown = owner_of_key(D, probe_key(w1, w2, wl));
    o.W = W;
    o.nid = K;
    o.iter = iter;
    o.tag = iter + 1;
    o.maxc = gm;
    o.ncand = nt;
    o.w1 = w1;
    o.w2 = w2;
    o.wl = wl;
    o.wfp = key_fp(W);
    if (D.kp_n) {  // the winner's posting list (per-key lists: tail.h / mid.h)
      o.kpn = solo ? pkn : ldc<COH>(&D.kp_n[W]);
      o.kpoff = solo ? pko : D.kp_off[W];
    }
    o.widL = L;
    o.wg = g;
    o.widR = Rr;
    publish();
  }
  dbg_stamp(D, 26);
}

// workgroup 0: the select; workgroups 1..: the previous merge's k_place (place != 0: it needs
// only k_commit's output) and, with the peer exchange (nimp > 0, exchange.h), first the import
// of the previous launch's records in workgroups 1..nimp, which the select waits for
__global__ __launch_bounds__(SBLOCK) void k_select(Dev D, int par, int run_end, int place, int nimp) {
  __shared__ int32_t s_red[SBLOCK / 64];
  __shared__ SelStage S;
  State* st = D.st;
  if (blockIdx.x > 0) {
    const int32_t b = blockIdx.x - 1;
    if (b < nimp) {
      __shared__ XImpLds X;
      x_import_share(D, X, b, nimp, false);
    }
    if (place && b < D.NBA) {
      __shared__ PlaceLds P;
      place_body(D, b, P);
    }
    return;
  }
  if (par == INT32_MIN) return;  // place only
  if (par < 0) {  // pipelined exchange: parity from the device's iteration count; no-op while stalled
    if (nimp > 0) {
      if (!x_import_wait(D, st->xpend != 0, nimp)) return;
    } else if (st->stall) {
      return;
    }
    const int32_t g = st->dgen + 1;
    par = g & 1;
    __syncthreads();  // every thread has read dgen
    if (threadIdx.x == 0) st->dgen = g;
  }
  __shared__ Sel s_sel;
  select_core<false>(D, par, S, s_red, &s_sel, run_end);
}

// merge replay (bin/induce.py): merge t is the trained
// token K0 + t, not the argmax.  Its key is looked up by content hash (find
// only); absent or at count 0 it merges nothing but still takes its token id.
// The posting index is rebuilt by the training rule (a rebuild iteration
// consumes no merge).  One thread: a few loads.
__global__ __launch_bounds__(64) void k_select_replay(Dev D, int par, const ReplayRec* fk, int64_t M) {
  if (threadIdx.x != 0) return;
  State* st = D.st;
  Sel* out = D.sel + par;
  const int32_t iter = st->iter, K = st->K;
  if (st->done || iter >= M) {
    out->decision = SEL_DONE;
    out->maxc = 0;
    return;
  }
  if (K >= D.KC) {
    set_error(D, GEOBPE_ECAPACITY, -9);
    out->decision = SEL_DONE;
    return;
  }
  const ReplayRec r = fk[iter];
  const u64 k = probe_key(r.h1, r.h2, r.len);
  const u64 mask = (u64)D.HC - 1;
  u64 s = ht_first_slot(D, k);
  int32_t W = -1;
  for (int64_t probe = 0; probe < D.HC; probe++) {
    const u64 cur = D.ht_key[s];
    if (cur == k) {
      W = (int32_t)s;
      break;
    }
    if (cur == 0) break;
    s = (s + 1) & mask;
  }
  if (W >= 0 && (D.kh1[W] != r.h1 || D.kh2[W] != r.h2 || D.klen[W] != r.len)) {
    set_error(D, GEOBPE_EHASH, iter);
    out->decision = SEL_DONE;
    return;
  }
  const int32_t c = W >= 0 ? D.count[W] : 0;
  if (c <= 0) W = -1;
  D.vh1[K] = r.h1;
  D.vh2[K] = r.h2;
  D.vlen[K] = r.len;
  LogRec lr;
  lr.nid = K;
  lr.count = c;
  lr.W = W;
  lr.idL = r.idL;
  lr.g = r.g;
  lr.idR = r.idR;
  lr.nmerged = 0;
  D.log[iter] = lr;
  out->decision = SEL_MERGE;
  out->skip = 0;
  out->rebuild = post_stale(D, c) ? 1 : 0;
  out->wown = owner_of_key(D, k);
  out->W = W;
  out->nid = K;
  out->iter = iter;
  out->tag = iter + 1;
  out->maxc = c;
  out->ncand = 1;
  out->w1 = r.h1;
  out->w2 = r.h2;
  out->wl = r.len;
  out->wfp = W >= 0 ? key_fp(W) : 0;
  out->widL = r.idL;
  out->wg = r.g;
  out->widR = r.idR;
}

// ====================================================================== multi-rank deltas
// merge events for the checkpoint's merge tree (TokenHierarchy / BinaryTreeBuilder.
// combine, data_structures.py:32-60, 217-226): after a merge iteration's k_commit,
// (merge index, left token start, right token start) of every merged occurrence
// from the find regions and the overflow list.  Record mode only (one launch per
// iteration); the hot kernels are unchanged.
__global__ __launch_bounds__(BLOCK) void k_events(Dev D, int par, int4* ev, int64_t cap, unsigned long long* ev_n) {
  __shared__ int64_t s_base;
  if (par < 0) {  // pipelined exchange (k_select set dgen)
    if (D.st->stall) return;
    par = D.st->dgen & 1;
  }
  const Sel sel = D.sel[par];
  if (sel.decision != SEL_MERGE) return;
  const int64_t novf = min(D.st->L_ovf2[par], D.Lovf_cap);
  const int64_t per = (novf + gridDim.x - 1) / gridDim.x;
  const int64_t o_lo = min(novf, (int64_t)blockIdx.x * per), o_hi = min(novf, o_lo + per);
  const int32_t nreg = blockIdx.x < D.NBA ? D.Lcnt[blockIdx.x] : 0;  // find region blockIdx.x
  if (threadIdx.x == 0) {
    const int64_t n = nreg + (o_hi - o_lo);
    s_base = n ? (int64_t)atomicAdd(ev_n, (unsigned long long)n) : 0;
  }
  __syncthreads();
  for (int32_t j = threadIdx.x; j < nreg; j += BLOCK) {
    const LEntry e = D.L[(int64_t)blockIdx.x * D.LC + j];
    if (s_base + j < cap) ev[s_base + j] = make_int4(sel.iter, e.a, e.b, 0);
  }
  for (int64_t k = o_lo + threadIdx.x; k < o_hi; k += BLOCK) {
    const LEntry e = D.Lovf[k];
    const int64_t at = s_base + nreg + (k - o_lo);
    if (at < cap) ev[at] = make_int4(sel.iter, e.a, e.b, 0);
  }
}

__global__ __launch_bounds__(BLOCK) void k_export(Dev D, DeltaRec* out, int64_t n) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    const int32_t d = D.touched[j];
    DeltaRec r;
    r.h1 = D.kh1[d];
    r.h2 = D.kh2[d];
    r.len = D.klen[d];
    r.idL = D.krep[3 * d];
    r.g = D.krep[3 * d + 1];
    r.idR = D.krep[3 * d + 2];
    r.delta = atomicExch(&D.dcount[d], 0);  // a key listed twice: the later copy carries 0
    r.pad = 0;
    out[j] = r;
  }
}

// device-counted export (no host round trip): every touched key's record, up to
// cap; k_export_fin then publishes the count and opens the next epoch
__global__ __launch_bounds__(BLOCK) void k_export_dev(Dev D, DeltaRec* out, int64_t cap, int chk_stall,
                                                     int64_t* d_count) {
  if (chk_stall && D.st->stall) return;  // pipelined: keep the stalled merge's records
  const int64_t nt = D.st->ntouched;
  const int64_t n = min(nt, cap);
  if (d_count && blockIdx.x == 0 && threadIdx.x == 0) {  // pipelined: the slot header (k_import_fixed resets ntouched)
    d_count[0] = nt;
    if (nt > cap) set_error(D, GEOBPE_ECAPACITY, -30);
  }
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    const int32_t d = D.touched[j];
    DeltaRec r;
    r.h1 = D.kh1[d];
    r.h2 = D.kh2[d];
    r.len = D.klen[d];
    r.idL = D.krep[3 * d];
    r.g = D.krep[3 * d + 1];
    r.idR = D.krep[3 * d + 2];
    r.delta = atomicExch(&D.dcount[d], 0);  // a key listed twice: the later copy carries 0
    r.pad = 0;
    out[j] = r;
  }
}
__global__ void k_export_fin(Dev D, int64_t* d_count, int64_t cap) {
  State* st = D.st;
  const int64_t n = st->ntouched;
  d_count[0] = n;
  if (n > cap) set_error(D, GEOBPE_ECAPACITY, -30);
  st->ntouched = 0;
  st->epoch += 1;  // every key may be touched again
}

__global__ __launch_bounds__(ABLOCK) void k_import(Dev D, const DeltaRec* in, int64_t n) {
  __shared__ int32_t s_np, s_ns;
  if (threadIdx.x == 0) s_np = s_ns = 0;
  __syncthreads();
  const int64_t E = (n + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * E, hi = min(n, lo + E);
  for (int64_t j = lo + threadIdx.x; j < hi; j += blockDim.x) {
    const DeltaRec r = in[j];
    if (r.delta == 0) continue;
    add_pair(D, &s_np, &s_ns, -1, r.h1, r.h2, r.len, r.idL, r.g, r.idR, r.delta);
  }
  close_regions(D, &s_np, &s_ns);
}

// pipelined exchange: the all-gathered fixed slots of `world` ranks, each
// {int64 count, pad to 40 B} + capf records.  A count above capf (that rank's
// records did not fit) stalls the pipeline instead: nothing is imported, and the
// host re-exchanges that merge's deltas in full (geobpe_pipeline_resolve).
// Import and finalize in one pass: every record's key is found or claimed and its
// delta added to the global count at once (the ranks' deltas are per key already;
// no LDS aggregation to gain), with the hot-list crossing check; a found key's
// content joins this workgroup's check region (verified by the next k_mark, as
// k_apply's finds are).  Also opens the next delta epoch (the export consumed it).
__global__ __launch_bounds__(ABLOCK) void k_import_fixed(Dev D, const uint8_t* in, int world, int64_t capf, int myrank,
                                                        int64_t* own_head) {
  __shared__ int32_t s_ns, s_chk, s_bad;
  __shared__ int64_t s_cnt[PIPE_MAX_WORLD + 1];
  __shared__ HotApp hot;
  State* st = D.st;
  if (st->stall) return;
  const int64_t slot = (1 + capf) * (int64_t)sizeof(DeltaRec);
  if (threadIdx.x == 0) {
    int64_t acc = 0, mx = 0;
    int bad = 0;
    for (int r = 0; r < world; r++) {
      const int64_t c = *reinterpret_cast<const int64_t*>(in + r * slot);
      s_cnt[r] = acc;
      acc += min(c, capf);
      mx = max(mx, c);
      bad |= c > capf;
    }
    s_cnt[world] = acc;
    s_bad = bad;
    s_ns = 0;
    s_chk = min(D.chkcnt[blockIdx.x], (int32_t)D.RC);  // after k_apply's finds
    if (blockIdx.x == 0) {
      st->slot_max = max(st->slot_max, mx);  // sizes the host's next slots (the poll resets it)
      st->ntouched = 0;   // the export of this merge consumed the touched list
      st->nxovf = 0;      // (k_commit turned k_find's side list into records)
      st->epoch += 1;
    }
  }
  hot_init(hot);
  __syncthreads();
  if (s_bad) {  // (this rank's slot header keeps the stalled merge's count for the full re-exchange)
    if (blockIdx.x == 0 && threadIdx.x == 0) st->stall = 1;
    return;
  }
  if (own_head && blockIdx.x == 0 && threadIdx.x == 0) *own_head = 0;  // (the middle regime counts into it)
  const int32_t th = st->theta;
  const int64_t n = s_cnt[world];
  const int64_t E = (n + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * E, hi = min(n, lo + E);
  for (int64_t j = lo + threadIdx.x; j < hi; j += blockDim.x) {
    int r = 0;
    while (j >= s_cnt[r + 1]) r++;
    const DeltaRec* recs = reinterpret_cast<const DeltaRec*>(in + r * slot + sizeof(DeltaRec));
    const DeltaRec rr = recs[j - s_cnt[r]];
    if (rr.delta == 0) continue;
    if (r == myrank && rr.pad > 0) {  // this rank's own record: its key id, resolved by k_commit
      count_add_hot(D, hot, rr.pad - 1, rr.delta, th);
      continue;
    }
    bool claimed;
    const int32_t d = ht_insert(D, rr.h1, rr.h2, rr.len, &claimed);
    if (d < 0) continue;
    if (claimed) {
      claim_payload(D, d, rr.h1, rr.h2, rr.len, rr.idL, rr.g, rr.idR);
      note_claim(D, &s_ns, d);
    } else {
      emit_check(D, &s_chk, d, rr.len, rr.h1, rr.h2);
    }
    count_add_hot(D, hot, d, rr.delta, th);
  }
  hot_flush(D, hot);
  close_claims(D, &s_ns);
  if (threadIdx.x == 0) D.chkcnt[blockIdx.x] = min(s_chk, (int32_t)D.RC);
}

// collapse of the row-sharded loop at the middle-regime switch (geobpe_run_exchange): every
// rank now holds every rank's token records, each block at its rank's residue base (rbase,
// W + 1 entries).  Links (tprev) move to global slots; a foreign block's pair keys are looked
// up again by content, in this rank's key table -- key ids are rank-local, and every rank
// holds every key (the exchange claimed each one on every rank, with its global count).
// A pair whose content is absent, or whose hashes differ from the key's, is an error.
__global__ __launch_bounds__(BLOCK) void k_collapse_fix(Dev D, const int64_t* rbase, int W, int own) {
  const u64 mask = (u64)D.HC - 1;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < D.R; g += (int64_t)gridDim.x * blockDim.x) {
    int r = 0;
    while (r + 1 < W && g >= rbase[r + 1]) r++;
    int4 t = D.tok[g];
    if (t.x < 0) continue;  // (not a token start)
    bool ch = false;
    if (t.z >= 0 && rbase[r]) {
      t.z += (int32_t)rbase[r];
      ch = true;
    }
    if (r != own && t.w >= 0) {
      const int32_t xlen = tok_len(t.y);
      const int64_t e = g + xlen - 1;
      const int4 te = D.tok[e + 1];  // (its x / y are never rewritten here)
      const int32_t gl = next_glue(D, t.y, e), ylen = tok_len(te.y);
      u64 h1, h2;
      combine(D, D.vh1[t.x], D.vh2[t.x], gl, D.vh1[te.x], D.vh2[te.x], ylen, h1, h2);
      const int32_t len = xlen + ylen;
      const u64 k = probe_key(h1, h2, len);
      u64 s = ht_first_slot(D, k);
      int32_t d = -1;
      for (int64_t probe = 0; probe < D.HC; probe++) {
        const u64 cur = D.ht_key[s];
        if (cur == k) {
          d = (int32_t)s;
          break;
        }
        if (cur == 0) break;
        s = (s + 1) & mask;
      }
      if (d < 0 || D.kh1[d] != h1 || D.kh2[d] != h2 || D.klen[d] != len) {
        set_error(D, d < 0 ? GEOBPE_ESTATE : GEOBPE_EHASH, g);
        d = -1;
      }
      t.w = d;
      ch = true;
    }
    if (ch) D.tok[g] = t;
  }
}

// ====================================================================== exports / checks
__global__ __launch_bounds__(BLOCK) void k_row_ntok(Dev D, int64_t* ntok) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < D.nrows; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = D.row_off[r], b = D.row_off[r + 1];
    int64_t n = 0;
    for (int64_t g = a; g < b; g += tok_len(D.tok[g].y)) n++;
    ntok[r] = n;
  }
}

__global__ __launch_bounds__(BLOCK) void k_row_seg(Dev D, const int64_t* tok_off, int32_t* start, int32_t* id) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < D.nrows; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = D.row_off[r], b = D.row_off[r + 1];
    int64_t t = tok_off[r];
    for (int64_t g = a; g < b;) {
      const int4 tg = D.tok[g];
      start[t] = (int32_t)(g - a);
      id[t] = tg.x;
      t++;
      g += tok_len(tg.y);
    }
  }
}

// quantize(tokenize()) per chain: id, then K+B+omega, K+2B+phi, K+cnca
// (tokenizer.py:379-392, bpe.py:918-956)
__global__ __launch_bounds__(BLOCK) void k_row_encode(Dev D, const int64_t* id_off, int32_t* ids, int32_t K) {
  const int32_t B = D.B;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < D.nrows; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = D.row_off[r], b = D.row_off[r + 1];
    int64_t t = id_off[r];
    for (int64_t g = a; g < b;) {
      const int4 tg = D.tok[g];
      const int64_t e = g + tok_len(tg.y) - 1;
      ids[t++] = tg.x;
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

// full recount of the live pair histogram from pk (verification)
__global__ __launch_bounds__(BLOCK) void k_recount(Dev D) {
  __shared__ Agg agg;
  agg_init(agg);
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < D.R; g += (int64_t)gridDim.x * blockDim.x) {
    const int32_t d = tok_pk(D, g);
    if (d >= 0 && !agg_stage(agg, d, 1)) atomicAdd(&D.scratch[d], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < Agg::N; i += blockDim.x)
    if (agg.key[i] >= 0) atomicAdd(&D.scratch[agg.key[i]], agg.val[i]);
}

// the number of keys (klist entries; chunk tails hold -1): counted when asked for, so
// no claim anywhere touches a shared key counter
__global__ __launch_bounds__(BLOCK) void k_count_keys(Dev D) {
  const int64_t U = min(D.st->U, D.KCAP);
  int32_t n = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < U; i += (int64_t)gridDim.x * blockDim.x)
    n += D.klist[i] >= 0;
  n = wave_sum(n);
  if (wave_lane() == 0 && n) atomicAdd((unsigned long long*)&D.st->nkeys, (unsigned long long)n);
}

__global__ __launch_bounds__(BLOCK) void k_compare(Dev D) {
  const int64_t U = min(D.st->U, D.KCAP);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < U; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t d = D.klist[i];
    if (d >= 0 && D.scratch[d] != D.count[d]) atomicAdd((unsigned long long*)&D.st->nmismatch, 1ULL);
  }
}

// debug: (key id, count) of every listed key
__global__ __launch_bounds__(BLOCK) void k_gather_counts(Dev D, int32_t* keys, int32_t* counts, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t d = D.klist[i];
    keys[i] = d;
    counts[i] = d >= 0 ? D.count[d] : 0;
  }
}

// debug: device key-string order of n (a, b) key pairs, one wave per pair: the
// char generator (key_less) and the wave comparator; 2 = they disagree
__global__ __launch_bounds__(256) void k_debug_key_less(Dev D, const int32_t* pairs, int32_t* out, int32_t n) {
  __shared__ char s_jbuf[48 * 256];
  const int32_t i = (int32_t)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (i >= n) return;  // wave-uniform
  const int32_t a = pairs[2 * i], b = pairs[2 * i + 1];
  const bool w = wave_key_less(key_seq(D, a), key_seq(D, b), D.B);
  if ((threadIdx.x & 63) == 0) {
    const bool j = key_less(D, a, b, s_jbuf + 48 * threadIdx.x);
    out[i] = j != w ? 2 : (j ? 1 : 0);
  }
}

#include "tail.h"
#include "mid.h"

}  // namespace gb
