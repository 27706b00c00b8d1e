// tail.h -- the late-merge path of BPE.step (foldingdiff/bpe.py:1792-2166).  Included
// once, by kernels.h, after k_select.
//
// Once the merges are small (a few thousand occurrences) the full-grid triple
// k_select -> k_find -> k_commit (+ k_place) is all latency: three launches, each a
// chain of cross-XCD round trips for ~2 k occurrences (~45-55 us a merge, DESIGN.md
// §8).  Here ONE workgroup of 1024 threads runs merge after merge in a single launch:
//
//   select   select_core (the same argmax + tie-break code as k_select)
//   find     the winner's own posting list (kpool[kp_off[W] ..]): one candidate per
//            thread, the greedy run walk of k_find (bpe.py:1888-1916)
//   commit   every new neighbour pair: key-table find-or-claim, +1 on its count (hot-list
//            crossing), an entry in its posting list; -1 on every destroyed pair
//   place    token rewrites and pk of the new pairs, after a barrier (the walks read the
//            pre-merge tokens)
//
// No other workgroup runs, so phases are separated by __syncthreads, not launches, and
// every round trip stays in this XCD's L2.  Reads of data this launch changes with
// atomics bypass the CU's L1 (ldc<true>).
//
// Posting lists: key d's list holds the token slots whose pair got key d since the last
// build (k_kp_*: a counting sort of the live pairs by key); a slot's pair only grows, so
// an entry is never listed twice, and entries whose token no longer carries d are
// skipped by the walk.  A list that runs out of capacity is regrown (2x) in the same
// merge; when the pool runs out the merge still completes, the lists are marked stale
// and the host rebuilds them before the next launch.
#pragma once
// (included inside namespace gb)

constexpr int TAIL_BIG = 256;      // regrown lists copied by the whole workgroup (LDS); more: rebuild
constexpr int TAIL_SMALL = 32;     // a regrown list of up to this capacity is copied by its own thread

struct TailLds {
  union {
    SelStage sel;
    struct {
      int32_t big_old[TAIL_BIG], big_new[TAIL_BIG], big_pre[TAIL_BIG + 1];
    } m;
  } u;
  Sel sel;
  HotApp hot;
  int32_t red[SBLOCK / 64];
  int32_t nM, nH, nS, nC, nrg, nbig, full;
};

struct TailCtx {
  int32_t W, nid, wl, th;
  u64 w1, w2;
  u64 pa1, pb1, pa2, pb2;  // P^(2 wl), P^(2 wl - 1) of both bases (a left key's right part is X)
};

// one reservation per wave instruction on a 64-bit global counter (the active lanes call it)
__device__ inline int64_t wave_reserve64(unsigned long long* ctr) {
  const u64 m = __ballot(1);
  const int lane = wave_lane();
  const int leader = __ffsll((long long)m) - 1;
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd(ctr, (unsigned long long)__popcll(m));
  base = __shfl(base, leader, 64);
  return (int64_t)(base + __popcll(m & ((1ULL << lane) - 1)));
}

// a new pair (idL, g, idR) of content hash (h1, h2), len residues, at token slot `target`:
// its key id (find or claim), +1 on its count, its posting entry; (slot, key) for the
// place phase
__device__ void tail_half(const Dev& D, TailLds& S, const TailCtx& F, u64 h1, u64 h2, int32_t len, int32_t idL,
                          int32_t g, int32_t idR, int32_t target) {
  bool claimed;
  const int32_t d = ht_insert(D, h1, h2, len, &claimed);
  if (d < 0) return;  // (capacity error set)
  if (claimed) {
    claim_payload(D, d, h1, h2, len, idL, g, idR);
    klist_put(D, wave_reserve64((unsigned long long*)&D.st->U), d);
  } else {
    const int32_t j = atomicAdd(&S.nC, 1);
    if (j < D.THcap) {
      NewPair e;
      e.target = d;
      e.slot = -1;
      e.len = len;
      e.delta = 0;
      e.h1 = h1;
      e.h2 = h2;
      D.TK[j] = e;
    }
  }
  const int32_t cap = D.kp_cap[d], off = D.kp_off[d];  // (changed only by the regrow phase)
  count_add_hot(D, S.hot, d, 1, F.th);
  const int32_t j = atomicAdd(&D.kp_n[d], 1);
  if (j < cap) {
    D.kpool[(int64_t)off + j] = target;
  } else {
    if (j == cap) {  // the list is regrown after the walks
      const int32_t r = atomicAdd(&S.nrg, 1);
      if (r < D.THcap) D.TR[r] = d;
    }
    const int32_t s = atomicAdd(&S.nS, 1);
    if (s < D.THcap) D.TS[s] = make_int4(d, j, target, 0);
  }
  const int32_t h = atomicAdd(&S.nH, 1);
  if (h < D.THcap) D.TH[h] = make_int2(target, d);
}

// the new key (X, glR, right) at slot t: right = X when the next token is a left part too
__device__ inline void tail_right(const Dev& D, TailLds& S, const TailCtx& F, int32_t t, int32_t glR, bool cL,
                                  int32_t idc, int32_t lc, u64 c1, u64 c2) {
  const int32_t rl = cL ? F.wl : lc;
  const u64 r1 = cL ? F.w1 : c1, r2 = cL ? F.w2 : c2;
  const int64_t ny = 2 * (int64_t)rl - 1;
  u64 h1, h2;
  combine_pw(F.w1, F.w2, glR, r1, r2, D.pw1[ny + 1], D.pw1[ny], D.pw2[ny + 1], D.pw2[ny], h1, h2);
  tail_half(D, S, F, h1, h2, F.wl + rl, F.nid, glR, cL ? F.nid : idc, t);
}

__device__ inline void tail_occ(const Dev& D, TailLds& S, int32_t a, int32_t ya, int32_t b, int32_t c) {
  const int32_t j = atomicAdd(&S.nM, 1);
  if (j < D.TMcap) D.TM[j] = make_int4(a, ya, b, c);
}

// candidate slot g of W: the walk of k_find (merge.h find_walk) with the commit work done
// in place -- the run start walks its run greedily left to right, every merged pair
// destroys its neighbours' pairs (-1) and makes the new ones
__device__ void tail_walk(const Dev& D, TailLds& S, const TailCtx& F, int32_t g) {
  const int32_t W = F.W;
  const int4 tg = D.tok[g];
  if (tg.w != W) return;  // (a stale entry: the token's pair changed since it was listed)
  const int32_t p = tg.z;
  const int32_t b = g + tok_len(tg.y);
  const int4 tp = D.tok[p >= 0 ? p : g];
  const int4 tb = D.tok[b];
  if (p >= 0 && tp.w == W) return;  // not a run start: its run's start walks it
  const int32_t glL = p >= 0 ? next_glue(D, tp.y, g - 1) : 0;
  const int32_t glR = next_glue(D, tb.y, g + F.wl - 1);
  const int32_t pkb = tb.w;
  const int32_t c = pkb >= 0 ? b + tok_len(tb.y) : -1;
  const int4 tc = D.tok[c >= 0 ? c : g];
  const int32_t pp = p >= 0 ? tp.z : -1;
  const int4 tpp = D.tok[pp >= 0 ? pp : g];
  const int32_t vp = p >= 0 ? max(tp.x, 0) : 0;
  const u64 l1 = D.vh1[vp], l2 = D.vh2[vp];
  const bool cL = c >= 0 && tc.w == W;
  const int32_t vc = c >= 0 ? max(tc.x, 0) : 0;
  const u64 c1 = D.vh1[vc], c2 = D.vh2[vc];
  bool pRight = false;
  if (p >= 0 && pp >= 0 && tpp.w == W) {  // the W-run ending at (pp, p): its length's parity
    int32_t m = 1, y = tpp.z;
    for (;;) {
      if (y < 0) break;
      const int4 ty = D.tok[y];
      if (ty.w != W) break;
      if (++m > D.R) {  // (a link cycle: report it instead of spinning)
        set_error(D, GEOBPE_ESTATE, y);
        break;
      }
      y = ty.z;
    }
    pRight = (m & 1) != 0;
  }
  const bool pN = p >= 0 && !pRight;
  tail_occ(D, S, g, F.wl | (tb.y & (int32_t)0xFFFF0000), b, c);
  if (pkb >= 0) atomicAdd(&D.count[pkb], -1);
  if (pN) {
    atomicAdd(&D.count[tp.w], -1);
    u64 h1, h2;
    combine_pw(l1, l2, glL, F.w1, F.w2, F.pa1, F.pb1, F.pa2, F.pb2, h1, h2);
    tail_half(D, S, F, h1, h2, tok_len(tp.y) + F.wl, tp.x, glL, F.nid, p);
  }
  if (c >= 0) tail_right(D, S, F, g, glR, cL, tc.x, tok_len(tc.y), c1, c2);
  // the rest of the run: (c, d) while (b, c) and (c, d) are both W
  int32_t cur_c = c, cur_pkb = pkb;
  bool cur_cL = cL;
  int32_t lcur_c = tok_len(tc.y);
  for (int64_t steps = 0; cur_pkb == W && cur_cL; steps++) {
    if (steps > D.R || lcur_c <= 0) {  // (a walk that does not advance: report it instead of spinning)
      set_error(D, GEOBPE_ESTATE, cur_c);
      break;
    }
    const int32_t t = cur_c;
    const int32_t b2 = t + lcur_c;
    const int4 tb2 = D.tok[b2];
    const int32_t glR2 = next_glue(D, tb2.y, t + F.wl - 1);
    const int32_t pkb2 = tb2.w;
    const int32_t c2i = pkb2 >= 0 ? b2 + tok_len(tb2.y) : -1;
    const int4 tc2 = D.tok[c2i >= 0 ? c2i : t];
    const bool cL2 = c2i >= 0 && tc2.w == W;
    const int32_t vc2 = c2i >= 0 ? max(tc2.x, 0) : 0;
    const u64 d1 = D.vh1[vc2], d2 = D.vh2[vc2];
    tail_occ(D, S, t, F.wl | (tb2.y & (int32_t)0xFFFF0000), b2, c2i);
    if (pkb2 >= 0) atomicAdd(&D.count[pkb2], -1);
    if (c2i >= 0) tail_right(D, S, F, t, glR2, cL2, tc2.x, tok_len(tc2.y), d1, d2);
    cur_c = c2i;
    cur_pkb = pkb2;
    cur_cL = cL2;
    lcur_c = tok_len(tc2.y);
  }
}

// up to n_max merges in one workgroup (grid 1, SBLOCK threads).  Stops early when an
// iteration is not a merge (hot-list rebuild or done: the host runs it with k_commit on
// parity st->tail_par), on an error, or after a merge whose posting lists went stale.
__global__ __launch_bounds__(SBLOCK) void k_tail(Dev D, int par, int64_t n_max) {
  __shared__ TailLds S;
  State* st = D.st;
  const int t = threadIdx.x;
  // EHASH check of the keys the last full-grid k_commit found (k_find would have done it)
  for (int32_t r = 0; r < D.NBA; r++) check_found(D, r);
  __syncthreads();
  if (t < D.NBA) D.chkcnt[t] = 0;
  if (t == 0) {
    st->place_par = -1;
    st->tail_exit = 0;
  }
  for (int64_t done = 0; done < n_max; done++) {
    if (ldc<true>(&st->err_code) != 0 || ldc<true>(&st->kp_valid) == 0) break;  // (uniform)
    select_core<true>(D, par, S.u.sel, S.red, &S.sel);
    __syncthreads();
    const int32_t decision = S.sel.decision;
    if (decision != SEL_MERGE) {
      if (t == 0) st->tail_exit = 1 + decision;
      break;
    }
    TailCtx F;
    F.W = S.sel.W;
    F.nid = S.sel.nid;
    F.wl = S.sel.wl;
    F.w1 = S.sel.w1;
    F.w2 = S.sel.w2;
    F.th = ldc<true>(&st->theta);
    const int32_t iter = S.sel.iter;
    {
      const int64_t nw = 2 * (int64_t)max(F.wl, 1) - 1;
      F.pa1 = D.pw1[nw + 1];
      F.pb1 = D.pw1[nw];
      F.pa2 = D.pw2[nw + 1];
      F.pb2 = D.pw2[nw];
    }
    {  // _tokens[n] = json.loads(key): content(L) ++ [g] ++ content(R)
      const int32_t L = S.sel.widL, g = S.sel.wg, Rr = S.sel.widR;
      const int64_t vL = D.voff[L], vR = D.voff[Rr];
      const int64_t nL = D.voff[L + 1] - vL, nR = D.voff[Rr + 1] - vR;
      const int64_t pos = D.voff[F.nid], ln = nL + 1 + nR;
      if (pos + ln > D.VSC) {
        if (t == 0) set_error(D, GEOBPE_ECAPACITY, -9);
      } else {
        for (int64_t i = t; i < ln; i += SBLOCK)
          D.vsym[pos + i] = i < nL ? D.vsym[vL + i] : (i == nL ? g : D.vsym[vR + i - nL - 1]);
        if (t == 0) D.voff[F.nid + 1] = pos + ln;
      }
    }
    if (t == 0) {
      S.nM = S.nH = S.nS = S.nC = S.nrg = S.nbig = S.full = 0;
      S.hot.n = 0;
    }
    __syncthreads();
    // ---- find + commit: the winner's posting list, one candidate per thread
    const int32_t nW = ldc<true>(&D.kp_n[F.W]);
    const int64_t offW = D.kp_off[F.W];
    for (int32_t c0 = 0; c0 < nW; c0 += SBLOCK) {
      const int32_t i = c0 + t;
      if (i < nW) {
        const int32_t g = D.kpool[offW + i];
        if (g >= 0 && g < D.R) tail_walk(D, S, F, g);  // (a bad list entry: no out-of-range read)
      }
    }
    __syncthreads();
    // ---- place: token rewrites (step 2, bond_to_token / token_pos) and pk of the new
    // pairs; the regrown lists' new space
    const int32_t nM = min(S.nM, (int32_t)D.TMcap), nH = min(S.nH, (int32_t)D.THcap);
    const int32_t nrg = min(S.nrg, (int32_t)D.THcap);
    if (S.nM > D.TMcap || S.nH > D.THcap) {
      if (t == 0) set_error(D, GEOBPE_ECAPACITY, -60);
    }
    for (int32_t i = t; i < nM; i += SBLOCK) {
      const int4 e = D.TM[i];
      *reinterpret_cast<int2*>(D.tok + e.x) = make_int2(F.nid, e.y);
      D.tok[e.z] = make_int4(-1, 0, -1, -1);
      if (e.w >= 0)
        *tok_f(D, e.w, 2) = e.x;
      else
        *tok_f(D, e.x, 3) = -1;
    }
    for (int32_t i = t; i < nH; i += SBLOCK) {
      const int2 h = D.TH[i];
      *tok_f(D, h.x, 3) = h.y;
    }
    // regrown lists (capacity 2n): space, the old entries (small lists by their thread, big
    // ones by the workgroup), then the entries past the old capacity
    bool stale = S.nrg > D.THcap || S.nS > D.THcap;
    if (!stale) {
      __shared__ int64_t s_base;
      for (int32_t r0 = 0; r0 < nrg; r0 += SBLOCK) {  // block-uniform rounds, one pool reservation each
        const int32_t r = r0 + t;
        int32_t d = -1, ncap = 0;
        if (r < nrg) {
          d = D.TR[r];
          ncap = max(2 * ldc<true>(&D.kp_n[d]), 16);
        }
        int32_t tot;
        const int32_t ex = block_excl_scan(ncap, &tot, S.red);
        if (t == 0) {
          s_base = (int64_t)atomicAdd((unsigned long long*)&st->kpool_used, (unsigned long long)tot);
          if (s_base + tot > D.KPOOL) S.full = 1;
        }
        __syncthreads();
        if (d >= 0 && !S.full) {
          const int64_t at = s_base + ex;
          const int32_t old = D.kp_off[d], cap = D.kp_cap[d];
          if (cap <= TAIL_SMALL) {
            for (int32_t k = 0; k < cap; k++) D.kpool[at + k] = D.kpool[(int64_t)old + k];
          } else {
            const int32_t q = atomicAdd(&S.nbig, 1);
            if (q < TAIL_BIG) {
              S.u.m.big_old[q] = old;
              S.u.m.big_new[q] = (int32_t)at;
              S.u.m.big_pre[q] = cap;
            } else {
              S.full = 1;
            }
          }
          D.kp_off[d] = (int32_t)at;
          D.kp_cap[d] = ncap;
        }
        __syncthreads();
      }
    }
    __syncthreads();
    stale = stale || S.full != 0;
    if (!stale && S.nbig > 0) {
      const int32_t nb = S.nbig;
      int32_t tc;
      const int32_t cx = block_excl_scan(t < nb ? S.u.m.big_pre[t] : 0, &tc, S.red);
      __syncthreads();
      if (t < nb) S.u.m.big_pre[t] = cx;
      if (t == 0) S.u.m.big_pre[nb] = tc;
      __syncthreads();
      for (int32_t q = t; q < tc; q += SBLOCK) {
        const int32_t r = seg_of(S.u.m.big_pre, nb, q);
        const int32_t k = q - S.u.m.big_pre[r];
        D.kpool[(int64_t)S.u.m.big_new[r] + k] = D.kpool[(int64_t)S.u.m.big_old[r] + k];
      }
    }
    if (!stale) {
      const int32_t nS = S.nS;
      for (int32_t i = t; i < nS; i += SBLOCK) {  // the entries past the old capacity
        const int4 e = D.TS[i];
        D.kpool[(int64_t)D.kp_off[e.x] + e.y] = e.z;
      }
    }
    if (stale && t == 0) st->kp_valid = 0;  // (this merge completes; the lists are rebuilt)
    // ---- EHASH check of the keys found; W's merged pairs; merge log and state
    const int32_t nC = min(S.nC, (int32_t)D.THcap);
    for (int32_t i = t; i < nC; i += SBLOCK) {
      const NewPair e = D.TK[i];
      const int32_t d = e.target;
      if (!key_is(D, d, e.h1, e.h2, e.len)) set_error(D, GEOBPE_EHASH, i);
    }
    if (D.ev) {  // merge events (record mode): (merge, left start, right start)
      __shared__ int64_t s_ev;
      if (t == 0) s_ev = nM ? (int64_t)atomicAdd(D.ev_n, (unsigned long long)nM) : 0;
      __syncthreads();
      for (int32_t i = t; i < nM; i += SBLOCK) {
        const int4 e = D.TM[i];
        if (s_ev + i < D.ev_cap) D.ev[s_ev + i] = make_int4(iter, e.x, e.z, 0);
      }
    }
    if (t == 0) {
      if (nM) atomicAdd(&D.count[F.W], -nM);
      D.log[iter].nmerged = nM;
      st->iter = iter + 1;
      st->K = F.nid + 1;
      st->maxc = S.sel.maxc;
      st->ncand = S.sel.ncand;
    }
    hot_flush(D, S.hot);  // (syncs the workgroup first)
    par ^= 1;
    __syncthreads();
  }
  if (t == 0) st->tail_par = par;
}

// ---- posting-list build: a counting sort of the live pairs by key
__global__ __launch_bounds__(BLOCK) void k_kp_reset(Dev D) {
  const int64_t U = min(D.st->U, D.KCAP);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < U; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t d = D.klist[i];
    if (d >= 0) {
      D.kp_n[d] = 0;
      D.kp_cap[d] = 0;
      D.kp_off[d] = 0;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) D.st->kpool_used = 0;
}

__global__ __launch_bounds__(BLOCK) void k_kp_count(Dev D) {
  __shared__ Agg agg;
  agg_init(agg);
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < D.R; g += (int64_t)gridDim.x * blockDim.x) {
    const int32_t d = tok_pk(D, g);
    if (d >= 0 && !agg_stage(agg, d, 1)) atomicAdd(&D.kp_n[d], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < Agg::N; i += blockDim.x)
    if (agg.key[i] >= 0) atomicAdd(&D.kp_n[agg.key[i]], agg.val[i]);
}

// list space: n + n/2 + 4 entries per key with live pairs (growth room), one pool
// reservation per round of the block.  from_count: n is the key's count (one rank: the
// count of a key IS its number of live pair slots, k_recount's invariant -- no counting
// pass); else k_kp_count's n (a rank's counts are global)
__global__ __launch_bounds__(BLOCK) void k_kp_alloc(Dev D, int from_count) {
  __shared__ int32_t s_red[BLOCK / 64];
  __shared__ int64_t s_base;
  const int64_t U = min(D.st->U, D.KCAP);
  const int64_t per = (U + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * per, hi = min(U, lo + per);
  for (int64_t i0 = lo; i0 < hi; i0 += BLOCK) {  // block-uniform
    const int64_t i = i0 + threadIdx.x;
    const int32_t d = i < hi ? D.klist[i] : -1;
    const int32_t n = d >= 0 ? max(from_count ? D.count[d] : D.kp_n[d], 0) : 0;
    const int32_t cap = n > 0 ? n + (n >> 1) + 4 : 0;
    int32_t tot;
    const int32_t ex = block_excl_scan(cap, &tot, s_red);
    if (threadIdx.x == 0) s_base = tot ? (int64_t)atomicAdd((unsigned long long*)&D.st->kpool_used, (unsigned long long)tot) : 0;
    __syncthreads();
    if (d >= 0) {
      if (s_base + ex + cap > D.KPOOL) set_error(D, GEOBPE_ECAPACITY, -61);
      D.kp_off[d] = (int32_t)(s_base + ex);
      D.kp_cap[d] = s_base + ex + cap > D.KPOOL ? 0 : cap;
      D.kp_n[d] = 0;
    }
    __syncthreads();
  }
}

// The lists' entries, one per live pair: a rank within its key from an atomic on the key's cursor.
// One returning atomic per pair serialised on the hottest keys' cursors at the memory side (the
// build ran ~50 ns a residue whatever the corpus: 1.54 ms at C3, 0.93 ms for half of it, in the
// merge loop at the middle-regime switch): the pairs of a round (KPF_U per thread) are grouped by
// key in LDS, each key takes its round's entries with ONE global atomic, and a pair's rank is its
// LDS rank after that base.  (A key's list order was never fixed: the atomics ordered it.)
constexpr int KPF_T = 512;   // threads
constexpr int KPF_U = 4;     // pairs per thread per round
constexpr int KPF_S = 4096;  // LDS key slots per round (>= 2x the round's pairs)
__global__ __launch_bounds__(KPF_T) void k_kp_fill(Dev D) {
  __shared__ int32_t skey[KPF_S], scnt[KPF_S], sbase[KPF_S];
  const int t = threadIdx.x;
  for (int i = t; i < KPF_S; i += KPF_T) {
    skey[i] = -1;
    scnt[i] = 0;
  }
  __syncthreads();
  constexpr int64_t ROUND = (int64_t)KPF_T * KPF_U;
  for (int64_t r0 = (int64_t)blockIdx.x * ROUND; r0 < D.R; r0 += (int64_t)gridDim.x * ROUND) {  // block-uniform
    int32_t d[KPF_U], s[KPF_U], rk[KPF_U];
#pragma unroll
    for (int u = 0; u < KPF_U; u++) {
      const int64_t g = r0 + t + (int64_t)u * KPF_T;
      d[u] = g < D.R ? tok_pk(D, g) : -1;
    }
#pragma unroll
    for (int u = 0; u < KPF_U; u++) {
      s[u] = -1;
      rk[u] = 0;
      if (d[u] < 0) continue;
      int32_t h = (int32_t)(((uint32_t)d[u] * 0x9E3779B1u) >> (32 - 12)) & (KPF_S - 1);
#pragma unroll 1
      for (int probe = 0; probe < 64; probe++, h = (h + 1) & (KPF_S - 1)) {
        int32_t c = skey[h];
        if (c == -1) c = atomicCAS(&skey[h], -1, d[u]);
        if (c == -1 || c == d[u]) {
          s[u] = h;
          rk[u] = atomicAdd(&scnt[h], 1);
          break;
        }
      }
    }
    __syncthreads();
    for (int i = t; i < KPF_S; i += KPF_T) {  // one cursor atomic per key of the round
      const int32_t k = skey[i];
      if (k >= 0) sbase[i] = atomicAdd(&D.kp_n[k], scnt[i]);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < KPF_U; u++) {
      if (d[u] < 0) continue;
      const int32_t j = s[u] >= 0 ? sbase[s[u]] + rk[u] : atomicAdd(&D.kp_n[d[u]], 1);  // (probes ran out: alone)
      if (j < D.kp_cap[d[u]]) D.kpool[(int64_t)D.kp_off[d[u]] + j] = (int32_t)(r0 + t + (int64_t)u * KPF_T);
    }
    for (int i = t; i < KPF_S; i += KPF_T) {  // (every thread has read its slots' bases above)
      if (skey[i] >= 0) {
        skey[i] = -1;
        scnt[i] = 0;
      }
    }
    __syncthreads();
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    D.st->kp_valid = 1;
    D.st->tail_exit = 0;
  }
}
