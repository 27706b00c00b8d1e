// bin_dense.h -- BPE.bin (bpe.py:1431-1474) at the initial state, where every
// token is one residue.  Included by kernels.h (after the key-table helpers).
//
// A pair's key content is then the symbol triple (left label, junction symbol,
// right label): the histogram needs no per-pair key probe.  The hot corner of
// the triple space is a "cube" of CL x CG x CL cells over the most frequent
// labels / junction symbols (<= 16384 cells: one LDS array), and the keys of
// its sampled cells are claimed BEFORE the count pass, so that pass writes the
// final pk of an in-cube pair directly and counts it with a plain LDS add.
// At C3 (B=5) the cube holds ~94 % of all pairs; the rest go to a per-workgroup
// list that a second, non-divergent kernel counts through an LDS hash table.
//
//   k_bin_sample   label / junction-symbol histograms of a 1/16 sample
//   k_bin_rank     (1 workgroup) frequency ranks; the cube shape maximising the
//                  sampled mass it covers; cube coordinate tables
//   k_bin_flag     cube cells that occur in the sample
//   k_bin_precube  each flagged cell claims its key (table slot = key id)
//   k_bin_count    the pass over every pair: 8 B in (tid, gsym), 4 B out (pk)
//                  for in-cube pairs; per-workgroup cube counts (LDS) ->
//                  one coalesced partial row per workgroup; the other pairs ->
//                  this workgroup's (slot, triple) list
//   k_bin_reduce   cube counts = sums of the partial rows
//   k_bin_ool      per list: LDS-staged counts per triple, one find-or-claim of
//                  each distinct triple's key, one count add, pk
//   k_bin_verify   every key a list found (not claimed) has this content
// The pair at residue slot g exists iff gsym[g] >= 0 (k_quantize: -1 = chain end).
#pragma once
// (inside namespace gb: kernels.h includes this file)

constexpr int BIN_VEC = 4;        // residue slots per int4 group
constexpr int BIN_GPT = 4;        // groups per thread per step (loads in flight together)
// (round 5 A/B: a count kernel that also wrote the merge loop's token records -- lane-strided
// 64-B record groups, 64 lines per store instruction -- took 287 us against 133 + a coalesced
// k_pack; the lean count kernel and k_pack stay)
constexpr int BIN_NC = 1 << 14;   // max cube cells (64 KB of LDS counts)
constexpr int BIN_SAMPLE = 16;    // the sample: the first 1/16 of each workgroup's range
constexpr int BIN_MAXSYM = 2048;  // label / junction-symbol tables (K0, B^3 <= 2048)
constexpr int BIN_RROWS = 32;     // partial rows summed per k_bin_reduce workgroup
using AggOol = AggT<13>;          // k_bin_ool: 8192 staged triples per list

// dense bin scratch (one allocation set per bin(); geobpe_bin)
struct BinWork {
  int32_t K0, G;
  int32_t nbc;            // count / list workgroups
  int32_t pad;
  int32_t* hist;          // [K0 + G] sampled label / junction-symbol counts
  int32_t* shape;         // [2] CL, CG
  int32_t* cl_of;         // [K0] cube coordinate of a label (-1: outside)
  int32_t* cg_of;         // [G]
  int32_t* l_at;          // [K0] label at cube coordinate r
  int32_t* g_at;          // [G]
  int32_t* flag;          // [BIN_NC] cell seen in the sample
  int32_t* cubemap;       // [BIN_NC] key id of a cube cell (-1: not pre-claimed)
  int32_t* partial;       // [nbc][BIN_NC] per-workgroup cube counts
  int2* ool;              // [nbc][ool_cap] (slot, triple) of out-of-cube pairs
  int32_t* ooln;          // [nbc]
  int2* found;            // [nbc][AggOol::N] (key id, triple) of keys a list found (sparse form)
  int32_t* foundn;        // [nbc]
  int64_t ool_cap;        // entries per list region
  int32_t* dcnt;          // [DS] dense form: count of an out-of-cube triple, then its key id
  int64_t DS;             // K0*G*K0 cells
  int32_t* newl;          // [newcap] dense form: triples counted for the first time
  unsigned long long* nnew;  // [1] entries of newl
  int64_t newcap;
};

__device__ inline int32_t bin_triple(int32_t la, int32_t gs, int32_t lb, int32_t G, int32_t K0) {
  return (la * G + gs) * K0 + lb;
}

// the next group's first token id: from the next lane by DPP (wave_shl:1, all
// lanes active); lane 63, and a lane whose next group is past its range, loads it
__device__ inline int32_t bin_next_tid(const Dev& D, int32_t tx, int64_t v, int64_t hi) {
  int32_t n = __builtin_amdgcn_update_dpp(-1, tx, 0x130, 0xF, 0xF, false);
  if ((wave_lane() == 63 || v + 1 >= hi) && v < hi) n = (v + 1) * BIN_VEC < D.R ? D.lab0[(v + 1) * BIN_VEC] : -1;
  return n;
}

// this workgroup's range of int4 groups (the count and sample passes agree on it)
__device__ inline void bin_range(const Dev& D, int64_t& lo, int64_t& hi) {
  const int64_t NV = D.R / BIN_VEC;
  const int64_t per = (NV + gridDim.x - 1) / gridDim.x;
  lo = (int64_t)blockIdx.x * per;
  hi = min(NV, lo + per);
}
__device__ inline int64_t bin_sample_end(int64_t lo, int64_t hi) {
  return min(hi, lo + (hi - lo + BIN_SAMPLE - 1) / BIN_SAMPLE);
}

__global__ __launch_bounds__(ABLOCK) void k_bin_sample(Dev D, BinWork W) {
  __shared__ int32_t h[2 * BIN_MAXSYM];
  const int32_t n = W.K0 + W.G;
  for (int i = threadIdx.x; i < n; i += ABLOCK) h[i] = 0;
  __syncthreads();
  int64_t lo, hi;
  bin_range(D, lo, hi);
  const int64_t he = bin_sample_end(lo, hi);
  const int4* tv = (const int4*)D.lab0;
  const int4* gv = (const int4*)D.gsym;
  for (int64_t v = lo + threadIdx.x; v < he; v += ABLOCK) {
    const int4 t = tv[v], s = gv[v];
    atomicAdd(&h[t.x], 1);
    atomicAdd(&h[t.y], 1);
    atomicAdd(&h[t.z], 1);
    atomicAdd(&h[t.w], 1);
    if (s.x >= 0) atomicAdd(&h[W.K0 + s.x], 1);
    if (s.y >= 0) atomicAdd(&h[W.K0 + s.y], 1);
    if (s.z >= 0) atomicAdd(&h[W.K0 + s.z], 1);
    if (s.w >= 0) atomicAdd(&h[W.K0 + s.w], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += ABLOCK)
    if (h[i]) atomicAdd(&W.hist[i], h[i]);
}

// rank of x[i] in decreasing count order (ties: smaller index first); x in LDS.
// One wave per element (lanes split the comparisons), so n <= 2048 costs
// n / 16 rounds of 32 LDS reads per lane.
__device__ inline void bin_ranks(const int32_t* x, int32_t n, int32_t* rank_of, int32_t* at_rank, double* mass) {
  const int lane = wave_lane();
  for (int32_t i = threadIdx.x >> 6; i < n; i += blockDim.x >> 6) {
    const int32_t xi = x[i];
    int32_t r = 0;
    for (int32_t j = lane; j < n; j += 64) r += x[j] > xi || (x[j] == xi && j < i);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o, 64);
    if (lane == 0) {
      rank_of[i] = r;
      at_rank[r] = i;
      mass[r] = (double)xi;
    }
  }
}

// in-place inclusive prefix sum of m[0..n) (n <= 2048) by one wave
__device__ inline void bin_cumsum(double* m, int32_t n) {
  const int lane = wave_lane();
  double carry = 0;
  for (int32_t b = 0; b < n; b += 64) {
    double x = b + lane < n ? m[b + lane] : 0.0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (b + lane < n) m[b + lane] = x + carry;
    carry += __shfl(x, 63, 64);
  }
}

__global__ __launch_bounds__(ABLOCK) void k_bin_rank(Dev D, BinWork W) {
  __shared__ double ml[BIN_MAXSYM], mg[BIN_MAXSYM];
  __shared__ int32_t x[2 * BIN_MAXSYM], rl[BIN_MAXSYM], rg[BIN_MAXSYM];
  __shared__ double s_best[ABLOCK];
  __shared__ int32_t s_cg[ABLOCK];
  const int32_t K0 = W.K0, G = W.G;
  for (int32_t i = threadIdx.x; i < K0 + G; i += ABLOCK) x[i] = W.hist[i];
  __syncthreads();
  bin_ranks(x, K0, rl, W.l_at, ml);
  bin_ranks(x + K0, G, rg, W.g_at, mg);
  __syncthreads();
  if (threadIdx.x < 64)
    bin_cumsum(ml, K0);
  else if (threadIdx.x < 128)
    bin_cumsum(mg, G);
  __syncthreads();
  // the shape with the largest covered (independence) mass: thread t tries CG = t+1, t+1+ABLOCK, ...
  double best = -1;
  int32_t bg = 1;
  for (int32_t cg = threadIdx.x + 1; cg <= G; cg += ABLOCK) {
    int32_t cl = (int32_t)sqrt((double)BIN_NC / cg);
    while (cl > 0 && cl * cl * cg > BIN_NC) cl--;
    while ((cl + 1) * (cl + 1) * cg <= BIN_NC) cl++;
    cl = min(cl, K0);
    if (cl < 1) continue;
    const double sc = ml[cl - 1] * ml[cl - 1] * mg[cg - 1];
    if (sc > best) {
      best = sc;
      bg = cg;
    }
  }
  s_best[threadIdx.x] = best;
  s_cg[threadIdx.x] = bg;
  __syncthreads();
  for (int o = ABLOCK / 2; o > 0; o >>= 1) {  // max (ties: smaller CG)
    if (threadIdx.x < o) {
      const double b2 = s_best[threadIdx.x + o];
      const int32_t g2 = s_cg[threadIdx.x + o];
      if (b2 > s_best[threadIdx.x] || (b2 == s_best[threadIdx.x] && g2 < s_cg[threadIdx.x])) {
        s_best[threadIdx.x] = b2;
        s_cg[threadIdx.x] = g2;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const int32_t cg = s_cg[0];
    int32_t cl = (int32_t)sqrt((double)BIN_NC / cg);
    while (cl > 0 && cl * cl * cg > BIN_NC) cl--;
    while ((cl + 1) * (cl + 1) * cg <= BIN_NC) cl++;
    s_cg[1] = min(max(cl, 1), K0);
    W.shape[0] = s_cg[1];
    W.shape[1] = cg;
  }
  __syncthreads();
  const int32_t CL = s_cg[1], CG = s_cg[0];
  for (int32_t i = threadIdx.x; i < K0; i += ABLOCK) W.cl_of[i] = rl[i] < CL ? rl[i] : -1;
  for (int32_t i = threadIdx.x; i < G; i += ABLOCK) W.cg_of[i] = rg[i] < CG ? rg[i] : -1;
}

// cube cell of a pair, or -1
__device__ inline int32_t bin_cell(const int32_t* cl, const int32_t* cg, int32_t CL, int32_t CG, int32_t la, int32_t gs,
                                   int32_t lb) {
  const int32_t a = cl[la], g = cg[gs], b = cl[lb];
  return (a | g | b) < 0 ? -1 : (a * CG + g) * CL + b;
}

__global__ __launch_bounds__(ABLOCK) void k_bin_flag(Dev D, BinWork W) {
  __shared__ int32_t cl[BIN_MAXSYM], cg[BIN_MAXSYM];
  __shared__ uint8_t f[BIN_NC];
  const int32_t CL = W.shape[0], CG = W.shape[1];
  for (int i = threadIdx.x; i < W.K0; i += ABLOCK) cl[i] = W.cl_of[i];
  for (int i = threadIdx.x; i < W.G; i += ABLOCK) cg[i] = W.cg_of[i];
  for (int i = threadIdx.x; i < BIN_NC; i += ABLOCK) f[i] = 0;
  __syncthreads();
  int64_t lo, hi;
  bin_range(D, lo, hi);
  const int64_t he = bin_sample_end(lo, hi);
  const int4* tv = (const int4*)D.lab0;
  const int4* gv = (const int4*)D.gsym;
  for (int64_t v = lo + threadIdx.x; v < he; v += ABLOCK) {
    const int4 t = tv[v], s = gv[v];
    // the three pairs inside the group (the 4th needs the next group's first token)
    int32_t c;
    if (s.x >= 0 && (c = bin_cell(cl, cg, CL, CG, t.x, s.x, t.y)) >= 0) f[c] = 1;
    if (s.y >= 0 && (c = bin_cell(cl, cg, CL, CG, t.y, s.y, t.z)) >= 0) f[c] = 1;
    if (s.z >= 0 && (c = bin_cell(cl, cg, CL, CG, t.z, s.z, t.w)) >= 0) f[c] = 1;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < CL * CG * CL; i += ABLOCK)
    if (f[i]) W.flag[i] = 1;
}

// the content hash of the residue pair (la, gs, lb)
__device__ inline void bin_hash(const Dev& D, int32_t la, int32_t gs, int32_t lb, u64& h1, u64& h2) {
  combine(D, D.vh1[la], D.vh2[la], gs, D.vh1[lb], D.vh2[lb], 1, h1, h2);
}

// claimed slots of one workgroup join klist with one reservation
constexpr int BIN_CLAIM_BUF = 8192;
struct ClaimBuf {
  int32_t n;
  int32_t slot[BIN_CLAIM_BUF];
};
__device__ inline void cb_init(ClaimBuf& cb) {
  if (threadIdx.x == 0) cb.n = 0;
  __syncthreads();
}
__device__ inline void cb_push(const Dev& D, ClaimBuf& cb, int32_t slot) {
  const int32_t j = atomicAdd(&cb.n, 1);
  if (j < BIN_CLAIM_BUF) {
    cb.slot[j] = slot;
  } else {  // rare: listed right away
    klist_put(D, (int64_t)atomicAdd((unsigned long long*)&D.st->U, 1ULL), slot);
  }
}
__device__ inline void cb_flush(const Dev& D, ClaimBuf& cb) {
  __shared__ int64_t s_base;
  __syncthreads();
  const int32_t n = min(cb.n, BIN_CLAIM_BUF);
  if (threadIdx.x == 0 && n) {
    s_base = (int64_t)atomicAdd((unsigned long long*)&D.st->U, (unsigned long long)n);
  }
  __syncthreads();
  for (int32_t j = threadIdx.x; j < n; j += blockDim.x) klist_put(D, s_base + j, cb.slot[j]);
}

// the sampled cube cells claim their keys (the first claims of the run: a found
// key here is a hash collision, GEOBPE_EHASH)
__global__ __launch_bounds__(BLOCK) void k_bin_precube(Dev D, BinWork W) {
  __shared__ ClaimBuf cb;
  cb_init(cb);
  const int32_t CL = W.shape[0], CG = W.shape[1];
  const int32_t nc = CL * CG * CL;
  const int32_t c = blockIdx.x * BLOCK + threadIdx.x;
  int32_t slot = -1;
  if (c < nc && W.flag[c]) {
    const int32_t b = c % CL, g = (c / CL) % CG, a = c / (CL * CG);
    const int32_t la = W.l_at[a], gs = W.g_at[g], lb = W.l_at[b];
    u64 h1, h2;
    bin_hash(D, la, gs, lb, h1, h2);
    bool claimed;
    slot = ht_insert(D, h1, h2, 2, &claimed);
    if (slot >= 0 && !claimed) {
      set_error(D, GEOBPE_EHASH, -10 - c);
      slot = -1;
    }
    if (slot >= 0) {
      claim_payload(D, slot, h1, h2, 2, la, gs, lb);
      cb_push(D, cb, slot);
    }
  }
  if (c < BIN_NC) W.cubemap[c] = slot;
  cb_flush(D, cb);
}

// a listed pair's key: the streamed pk that k_pack copies into the token record
__device__ inline void bin_set_pk(const Dev& D, int64_t g, int32_t k) { D.pk[g] = k; }

// a pair of k_bin_count outside the pre-claimed cube: this workgroup's list
__device__ inline void bin_list(const BinWork& W, int32_t* s_nool, int2* ool, int32_t la, int32_t gs, int32_t lb,
                                int64_t g) {
  const int32_t j = atomicAdd(s_nool, 1);
  if (j < W.ool_cap) ool[j] = make_int2((int32_t)g, bin_triple(la, gs, lb, W.G, W.K0));
}

// the pass over every pair.  LDS: the cube's key ids and counts, the cube
// coordinate tables; the out-of-cube pairs go to this workgroup's list region.
// Per step a thread's 16 pairs go through the LDS in batches (coordinates of all
// 20 tokens / 16 junctions, then 16 cube-map reads, then the adds), so each
// batch costs one LDS round trip, not one per pair.
__global__ __launch_bounds__(ABLOCK) void k_bin_count(Dev D, BinWork W) {
  __shared__ int32_t s_map[BIN_NC], s_cnt[BIN_NC];
  __shared__ int32_t cl[BIN_MAXSYM], cg[BIN_MAXSYM];
  __shared__ int32_t s_nool;
  const int32_t CL = W.shape[0], CG = W.shape[1], K0 = W.K0, G = W.G;
  const int32_t nc = CL * CG * CL;
  for (int i = threadIdx.x; i < nc; i += ABLOCK) {
    s_map[i] = W.cubemap[i];
    s_cnt[i] = 0;
  }
  for (int i = threadIdx.x; i < K0; i += ABLOCK) cl[i] = W.cl_of[i];
  for (int i = threadIdx.x; i < G; i += ABLOCK) cg[i] = W.cg_of[i];
  if (threadIdx.x == 0) s_nool = 0;
  __syncthreads();
  int64_t lo, hi;
  bin_range(D, lo, hi);
  const int64_t R = D.R;
  const int4* tv = (const int4*)D.lab0;
  const int4* gv = (const int4*)D.gsym;
  int4* pv = (int4*)D.pk;
  int2* ool = W.ool + (int64_t)blockIdx.x * W.ool_cap;
  for (int64_t v0 = lo; v0 < hi; v0 += BIN_GPT * ABLOCK) {
    int32_t ts[BIN_GPT][BIN_VEC + 1], ss[BIN_GPT][BIN_VEC];
#pragma unroll
    for (int q = 0; q < BIN_GPT; q++) {
      const int64_t v = v0 + q * ABLOCK + threadIdx.x;
      const int4 t = v < hi ? tv[v] : make_int4(0, 0, 0, 0);
      const int4 s = v < hi ? gv[v] : make_int4(-1, -1, -1, -1);
      ts[q][0] = t.x;
      ts[q][1] = t.y;
      ts[q][2] = t.z;
      ts[q][3] = t.w;
      ss[q][0] = s.x;
      ss[q][1] = s.y;
      ss[q][2] = s.z;
      ss[q][3] = s.w;
    }
#pragma unroll
    for (int q = 0; q < BIN_GPT; q++) {
      const int64_t v = v0 + q * ABLOCK + threadIdx.x;
      const int32_t nx = bin_next_tid(D, ts[q][0], v, hi);
      ts[q][BIN_VEC] = ss[q][BIN_VEC - 1] >= 0 ? nx : 0;
    }
    int32_t a[BIN_GPT][BIN_VEC + 1], c[BIN_GPT][BIN_VEC];
#pragma unroll
    for (int q = 0; q < BIN_GPT; q++) {
#pragma unroll
      for (int u = 0; u <= BIN_VEC; u++) a[q][u] = cl[ts[q][u]];
#pragma unroll
      for (int u = 0; u < BIN_VEC; u++) c[q][u] = ss[q][u] >= 0 ? cg[ss[q][u]] : -1;
    }
#pragma unroll
    for (int q = 0; q < BIN_GPT; q++)
#pragma unroll
      for (int u = 0; u < BIN_VEC; u++)
        c[q][u] = (a[q][u] | c[q][u] | a[q][u + 1]) < 0 ? -1 : (a[q][u] * CG + c[q][u]) * CL + a[q][u + 1];
    int32_t k[BIN_GPT][BIN_VEC];
#pragma unroll
    for (int q = 0; q < BIN_GPT; q++)
#pragma unroll
      for (int u = 0; u < BIN_VEC; u++) k[q][u] = c[q][u] >= 0 ? s_map[c[q][u]] : -1;
#pragma unroll
    for (int q = 0; q < BIN_GPT; q++) {
      const int64_t v = v0 + q * ABLOCK + threadIdx.x;
#pragma unroll
      for (int u = 0; u < BIN_VEC; u++) {
        if (k[q][u] >= 0)
          atomicAdd(&s_cnt[c[q][u]], 1);
        else if (ss[q][u] >= 0)
          bin_list(W, &s_nool, ool, ts[q][u], ss[q][u], ts[q][u + 1], v * BIN_VEC + u);
      }
      if (v < hi) pv[v] = make_int4(k[q][0], k[q][1], k[q][2], k[q][3]);
    }
  }
  if (blockIdx.x == gridDim.x - 1) {  // the < 4 slots past the last full group
    for (int64_t g = (R / BIN_VEC) * BIN_VEC + threadIdx.x; g < R; g += ABLOCK) {
      const int32_t sy = D.gsym[g];
      int32_t k = -1;
      if (sy >= 0) {
        const int32_t la = D.lab0[g], lb = D.lab0[g + 1];
        const int32_t cc = bin_cell(cl, cg, CL, CG, la, sy, lb);
        k = cc >= 0 ? s_map[cc] : -1;
        if (k >= 0)
          atomicAdd(&s_cnt[cc], 1);
        else
          bin_list(W, &s_nool, ool, la, sy, lb, g);
      }
      D.pk[g] = k;
    }
  }
  __syncthreads();
  int32_t* part = W.partial + (int64_t)blockIdx.x * BIN_NC;
  for (int i = threadIdx.x; i < nc; i += ABLOCK) part[i] = s_cnt[i];
  if (threadIdx.x == 0) {
    W.ooln[blockIdx.x] = min(s_nool, (int32_t)W.ool_cap);
    if (s_nool > W.ool_cap) set_error(D, GEOBPE_ECAPACITY, -20);
  }
}

// cube counts: sums of the partial rows.  Workgroup (x, y) adds rows
// [y*BIN_RROWS, (y+1)*BIN_RROWS) of cells [x*ABLOCK, (x+1)*ABLOCK).
__global__ __launch_bounds__(ABLOCK) void k_bin_reduce(Dev D, BinWork W, int to_delta) {
  const int32_t CL = W.shape[0], CG = W.shape[1];
  const int32_t nc = CL * CG * CL;
  const int32_t c = blockIdx.x * ABLOCK + threadIdx.x;
  if (c >= nc) return;
  const int32_t slot = W.cubemap[c];
  if (slot < 0) return;
  const int32_t w0 = blockIdx.y * BIN_RROWS, w1 = min(W.nbc, w0 + BIN_RROWS);
  int32_t part[BIN_RROWS];
#pragma unroll
  for (int i = 0; i < BIN_RROWS; i++) part[i] = w0 + i < w1 ? W.partial[(int64_t)(w0 + i) * BIN_NC + c] : 0;
  int32_t sum = 0;
#pragma unroll
  for (int i = 0; i < BIN_RROWS; i++) sum += part[i];
  if (sum) global_add(D, slot, sum, to_delta != 0);
}

// ---- the lists, dense form (K0 * B^3 * K0 <= 2^26 cells): a global count per
// triple.  k_bin_ool_stage: LDS-staged counts per list, one atomic per
// (list, triple); the add that finds a cell at 0 lists the triple as new.
// k_bin_ool_claim: one thread per new triple claims its key (a found key is a
// hash collision: every other bin key is a distinct triple).  k_bin_ool_fix: pk
// of every listed pair from the cell (now the key id).
__device__ inline void bin_stage_list(const Dev& D, AggOol& agg, int2* ool, int32_t n) {
  for (int32_t j = threadIdx.x; j < n; j += ABLOCK) {
    const int32_t d = ool[j].y;
    if (!agg_stage(agg, d, 1)) ool[j].y = -2 - d;  // LDS full: counted by the fix-up list itself
  }
  __syncthreads();
}

__global__ __launch_bounds__(ABLOCK) void k_bin_ool_stage(Dev D, BinWork W) {
  __shared__ AggOol agg;
  __shared__ int32_t s_nn;
  __shared__ int32_t s_new[AggOol::N];
  __shared__ int64_t s_base;
  agg_init(agg);
  if (threadIdx.x == 0) s_nn = 0;
  const int32_t n = W.ooln[blockIdx.x];
  const int2* ool = W.ool + (int64_t)blockIdx.x * W.ool_cap;
  __syncthreads();
  for (int32_t j = threadIdx.x; j < n; j += ABLOCK) {
    const int32_t d = ool[j].y;
    if (!agg_stage(agg, d, 1) && atomicAdd(&W.dcnt[d], 1) == 0) {  // LDS full (rare): straight to the cell
      const int64_t k = (int64_t)atomicAdd(&W.nnew[0], 1ULL);
      if (k < W.newcap) W.newl[k] = d;
    }
  }
  __syncthreads();
  for (int32_t h = threadIdx.x; h < AggOol::N; h += ABLOCK) {
    const int32_t d = agg.key[h];
    if (d >= 0 && atomicAdd(&W.dcnt[d], agg.val[h]) == 0) s_new[atomicAdd(&s_nn, 1)] = d;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    s_base = s_nn ? (int64_t)atomicAdd(&W.nnew[0], (unsigned long long)s_nn) : 0;
  __syncthreads();
  for (int32_t j = threadIdx.x; j < s_nn; j += ABLOCK)
    if (s_base + j < W.newcap) W.newl[s_base + j] = s_new[j];
}

__global__ __launch_bounds__(BLOCK) void k_bin_ool_claim(Dev D, BinWork W, int to_delta) {
  __shared__ ClaimBuf cb;
  cb_init(cb);
  const int64_t n = min((int64_t)W.nnew[0], W.newcap);
  const int32_t K0 = W.K0, G = W.G;
  for (int64_t j = (int64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLOCK) {
    const int32_t d = W.newl[j];
    const int32_t lb = d % K0, gs = (d / K0) % G, la = d / (K0 * G);
    u64 h1, h2;
    bin_hash(D, la, gs, lb, h1, h2);
    bool claimed;
    int32_t slot = ht_insert(D, h1, h2, 2, &claimed);
    if (slot >= 0 && !claimed) {
      set_error(D, GEOBPE_EHASH, d);
      slot = -1;
    }
    if (slot < 0) continue;
    claim_payload(D, slot, h1, h2, 2, la, gs, lb);
    cb_push(D, cb, slot);
    global_add(D, slot, W.dcnt[d], to_delta != 0);
    W.dcnt[d] = slot;
  }
  cb_flush(D, cb);
  if (blockIdx.x == 0 && threadIdx.x == 0 && W.nnew[0] > (unsigned long long)W.newcap)
    set_error(D, GEOBPE_ECAPACITY, -21);
}

__global__ __launch_bounds__(ABLOCK) void k_bin_ool_fix(Dev D, BinWork W) {
  const int32_t n = W.ooln[blockIdx.x];
  const int2* ool = W.ool + (int64_t)blockIdx.x * W.ool_cap;
  for (int32_t j = threadIdx.x; j < n; j += ABLOCK) {
    const int2 e = ool[j];
    const int32_t k = W.dcnt[e.y];
    bin_set_pk(D, e.x, k);
  }
}

// ---- the lists, sparse form (larger triple spaces): per list, LDS-staged counts
// per triple, then one find-or-claim and one count add per distinct triple,
// then pk of every listed pair.  A list holding more than AggOol::N
// distinct triples sends the rest through the key table one by one.
__global__ __launch_bounds__(ABLOCK) void k_bin_ool(Dev D, BinWork W, int to_delta) {
  __shared__ AggOol agg;
  __shared__ int32_t s_id[AggOol::N];
  __shared__ ClaimBuf cb;
  __shared__ int32_t s_nf;
  agg_init(agg);
  cb_init(cb);
  if (threadIdx.x == 0) s_nf = 0;
  const int32_t n = W.ooln[blockIdx.x];
  int2* ool = W.ool + (int64_t)blockIdx.x * W.ool_cap;
  int2* found = W.found + (int64_t)blockIdx.x * AggOol::N;
  const int32_t K0 = W.K0, G = W.G;
  __syncthreads();
  for (int32_t j = threadIdx.x; j < n; j += ABLOCK) {
    const int2 e = ool[j];
    uint32_t h = AggOol::slot(e.y);
    int32_t at = -1;
#pragma unroll 1
    for (int probe = 0; probe < 8; probe++) {
      int32_t k = agg.key[h];
      if (k == -1) k = atomicCAS(&agg.key[h], -1, e.y) == -1 ? e.y : agg.key[h];
      if (k == e.y) {
        atomicAdd(&agg.val[h], 1);
        at = (int32_t)h;
        break;
      }
      h = (h + 1) & (AggOol::N - 1);
    }
    if (at < 0) {  // LDS table full: this pair alone
      const int32_t lb = e.y % K0, gs = (e.y / K0) % G, la = e.y / (K0 * G);
      u64 h1, h2;
      bin_hash(D, la, gs, lb, h1, h2);
      bool claimed;
      const int32_t slot = ht_insert(D, h1, h2, 2, &claimed);
      if (slot >= 0) {
        if (claimed) {
          claim_payload(D, slot, h1, h2, 2, la, gs, lb);
          cb_push(D, cb, slot);
        } else {
          const int32_t f = atomicAdd(&s_nf, 1);
          if (f < AggOol::N) found[f] = make_int2(slot, e.y);
        }
        global_add(D, slot, 1, to_delta != 0);
      }
      bin_set_pk(D, e.x, slot);
      ool[j].y = -1;
    } else {
      ool[j].y = at;
    }
  }
  __syncthreads();
  for (int32_t h = threadIdx.x; h < AggOol::N; h += ABLOCK) {
    const int32_t d = agg.key[h];
    int32_t slot = -1;
    if (d >= 0) {
      const int32_t lb = d % K0, gs = (d / K0) % G, la = d / (K0 * G);
      u64 h1, h2;
      bin_hash(D, la, gs, lb, h1, h2);
      bool claimed;
      slot = ht_insert(D, h1, h2, 2, &claimed);
      if (slot >= 0) {
        if (claimed) {
          claim_payload(D, slot, h1, h2, 2, la, gs, lb);
          cb_push(D, cb, slot);
        } else {
          const int32_t f = atomicAdd(&s_nf, 1);
          if (f < AggOol::N) found[f] = make_int2(slot, d);
        }
        global_add(D, slot, agg.val[h], to_delta != 0);
      }
    }
    s_id[h] = slot;
  }
  __syncthreads();
  for (int32_t j = threadIdx.x; j < n; j += ABLOCK) {
    const int2 e = ool[j];
    if (e.y < 0) continue;
    const int32_t k = s_id[e.y];
    bin_set_pk(D, e.x, k);
  }
  cb_flush(D, cb);
  if (threadIdx.x == 0) {
    W.foundn[blockIdx.x] = min(s_nf, (int32_t)AggOol::N);
    if (s_nf > AggOol::N) atomicAdd((unsigned long long*)&D.st->nunchecked, (unsigned long long)(s_nf - AggOol::N));
  }
}

// a key found (not claimed) by a list must hold that list's content
__global__ __launch_bounds__(ABLOCK) void k_bin_verify(Dev D, BinWork W) {
  const int32_t n = W.foundn[blockIdx.x];
  const int2* found = W.found + (int64_t)blockIdx.x * AggOol::N;
  const int32_t K0 = W.K0, G = W.G;
  for (int32_t j = threadIdx.x; j < n; j += ABLOCK) {
    const int2 e = found[j];
    const int32_t lb = e.y % K0, gs = (e.y / K0) % G, la = e.y / (K0 * G);
    u64 h1, h2;
    bin_hash(D, la, gs, lb, h1, h2);
    if (D.kh1[e.x] != h1 || D.kh2[e.x] != h2 || D.klen[e.x] != 2) set_error(D, GEOBPE_EHASH, e.y);
  }
}
