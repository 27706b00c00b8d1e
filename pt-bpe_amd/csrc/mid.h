// mid.h -- the middle regime of BPE.step (foldingdiff/bpe.py:1792-2166): merges of up to
// a few thousand occurrences, on the per-key posting lists of tail.h.  Included once, by
// kernels.h, after tail.h.
//
// Two launches per merge t:
//   k_mid_sel   workgroup 0: select_core (argmax + reference tie-break), which also hands
//               the winner's list bounds to the find; workgroups 1..P: merge t-1's token
//               rewrites and pk of its new pairs, and the EHASH check of the keys its find
//               found (the select is the longer of the two)
//   k_mid_find  workgroups 0..G-1: find + commit of merge t -- the winner's candidates are
//               its posting list plus merge t-1's new pairs of its key, split over the
//               workgroups; the greedy run walks of k_find; the new pairs' keys deduplicated
//               per round in LDS and resolved once per (workgroup, key): find-or-claim,
//               +n on the count (hot-list crossing); -1 on the destroyed pairs
//               (LDS-aggregated); merged occurrences and new pairs to global lists.
//               Workgroups G..G+A-1: merge t-1's posting entries, each owning the keys of
//               one hash bucket (no cross-workgroup allocation: a full list grows 2x by its
//               owner).  The winner's own key is skipped: its pairs are being merged now
//               (all of them: its count drops to 0), which is why the find reads them from
//               the new-pair list instead.
// So the list appends run beside the find, off the path from one merge to the next.
// Compared with the full-grid find/commit/place (merge.h) there is no owner hand-off (key
// records, decrement records, posting logs): the per-key lists make the candidates exact
// and a late merge's keys are few per workgroup.
#pragma once
// (included inside namespace gb)

constexpr int MKC = 1024;   // k_mid_find: new-key dedupe slots per round (LDS)
constexpr int MPK = 2048;   // appends: key grouping slots (LDS)
constexpr int MID_APP = 32; // appending workgroups of k_mid_find (hash buckets of the keys)

__device__ inline int2* mid_th(const Dev& D, int par) { return D.TH + (int64_t)par * D.THcap; }
__device__ inline int32_t mid_G(const Dev& D) { return D.NBA - MID_APP; }  // find workgroups

constexpr int MTM = 1024;  // k_mid_find: merged occurrences buffered per workgroup (LDS)
constexpr int MTH = 2048;  // new pairs buffered per workgroup
constexpr int MKL = 1024;  // claimed keys buffered per workgroup
// The merged occurrences (TM) and new pairs (TH, per parity) of find workgroup w live in a
// fixed segment [w * MTM, + D.mcnt[par][w].x) / [w * MTH, + .y) -- written without any
// shared counter -- and past the segments in a spill list (st->mid_nm / mid_nh count it)
// for what did not fit the LDS buffer
constexpr int64_t MSEG_TM = (int64_t)NBA_MAX * MTM;
constexpr int64_t MSEG_TH = (int64_t)NBA_MAX * MTH;

struct MidFindLds {
  u64 key[MKC], h1[MKC], h2[MKC];
  int4 rep[MKC];  // {len, idL, g, idR}
  int32_t cnt[MKC], did[MKC];
  int32_t occ[MKC];  // occupied slots, in insertion order
  AggT<11> agg;      // count decrements
  HotApp hot;
  // the workgroup's list appends (merged occurrences, new pairs, claimed keys), written out
  // behind one reservation each when the find ends -- a reservation per wave instruction
  // on the shared counters put a returning global atomic on the walk's and the resolve's
  // paths (past the buffers: the per-wave path)
  int4 tm[MTM];
  int2 th[MTH];
  int32_t kl[MKL];
  int32_t bcnt[MID_APP + 1];  // the new pairs per appending workgroup, then their runs' starts
  int32_t red[ABLOCK / 64];
  int32_t nocc, nm, chk, ntm, nth, nkl;
  int64_t xbase, bk;
};
static_assert(MTH <= 2 * ABLOCK, "mid_flush_lists: two new pairs per thread");

constexpr int MAE = 6144;  // appends: this bucket's entries kept from pass 1 (LDS)
static_assert(MPK <= 2048, "an append entry packs its key slot in 11 bits");

struct MidAppLds {
  int32_t key[MPK], cnt[MPK], base[MPK], cur[MPK], off[MPK];
  int32_t occ[MPK];
  int2 ent[MAE];  // this bucket's new pairs {slot, key}, then {slot, key slot << 21 | rank (as uint32)}
  int32_t big_old[TAIL_BIG], big_new[TAIL_BIG], big_pre[TAIL_BIG + 1];
  int32_t pre[NBA_MAX + 1];  // prefix of this bucket's run lengths over the find workgroups' TH segments
  int32_t rb[NBA_MAX];       // this bucket's run start in each segment
  int32_t red[ABLOCK / 64];
  int32_t nocc, nbig, full, nent;
  int64_t pbase;
};

// ---------------------------------------------------------------------- find
struct MidCtx {
  int32_t W, nid, wl, th, par, iter, maxc;
  u64 w1, w2;
  u64 pa1, pb1, pa2, pb2;
};

// the appending workgroup (of A) that takes key d's posting entries
__device__ inline uint32_t mid_bucket(int32_t d, int32_t A) {
  return (uint32_t)(((u64)((uint32_t)d * 2654435761u) * (u64)A) >> 32);
}

// one LDS slot per active lane, one LDS atomic per wave instruction
__device__ inline int32_t lds_reserve(int32_t* n) {
  const u64 m = __ballot(1);
  const int lane = wave_lane();
  const int leader = __ffsll((long long)m) - 1;
  int32_t base = 0;
  if (lane == leader) base = atomicAdd(n, __popcll(m));
  base = __shfl(base, leader, 64);
  return base + __popcll(m & ((1ULL << lane) - 1));
}

__device__ inline void mid_occ(const Dev& D, MidFindLds& S, const MidCtx& F, int32_t a, int32_t ya, int32_t b,
                               int32_t c) {
  const int32_t k = lds_reserve(&S.ntm);
  if (k < MTM) {
    S.tm[k] = make_int4(a, ya, b, c);
  } else {
    const int64_t j = MSEG_TM + wave_reserve64((unsigned long long*)&D.st->mid_nm[F.par]);
    if (j < D.TMcap)
      D.TM[j] = make_int4(a, ya, b, c);
    else
      set_error(D, GEOBPE_ECAPACITY, -70);
  }
  atomicAdd(&S.nm, 1);
  if (D.ev) {  // merge events (record mode): (merge, left start, right start)
    const int64_t k = wave_reserve64(D.ev_n);
    if (k < D.ev_cap) D.ev[k] = make_int4(F.iter, a, b, 0);
  }
}

__device__ inline void mid_pair(const Dev& D, MidFindLds& S, const MidCtx& F, int32_t target, int32_t d) {
  const int32_t k = lds_reserve(&S.nth);
  if (k < MTH) {
    S.th[k] = make_int2(target, d);
    return;
  }
  const int64_t j = MSEG_TH + wave_reserve64((unsigned long long*)&D.st->mid_nh[F.par]);
  if (j < D.THcap)
    mid_th(D, F.par)[j] = make_int2(target, d);
  else
    set_error(D, GEOBPE_ECAPACITY, -71);
}

// a key this workgroup claimed joins klist
__device__ inline void mid_claimed(const Dev& D, MidFindLds& S, int32_t d) {
  const int32_t k = lds_reserve(&S.nkl);
  if (k < MKL) {
    S.kl[k] = d;
    return;
  }
  klist_put(D, wave_reserve64((unsigned long long*)&D.st->U), d);
}

// the buffered appends out (block-uniform): TM / TH into this workgroup's segments and the
// counts beside them, the claimed keys from this workgroup's klist chunk (a reservation only
// when the chunk runs out) -- no shared counter, so the find workgroups ending together do not
// queue on one address
__device__ inline void mid_flush_lists(const Dev& D, MidFindLds& S, int par, int32_t w, int64_t kc0, int64_t kc1) {
  State* st = D.st;
  const int32_t t = threadIdx.x;
  __syncthreads();
  const int32_t a = min(S.ntm, MTM), b = min(S.nth, MTH), c = min(S.nkl, MKL);
  if (t == 0) {
    D.mcnt[par * NBA_MAX + w] = make_int4(a, b, S.nm, 0);
    if (c) {  // (the chunk state came with the launch's first loads: no round trip here)
      int64_t k0 = kc0, k1 = kc1;
      if (k1 - k0 < c) {
        const int64_t sz = max((int64_t)KL_CHUNK, (int64_t)c);
        k0 = (int64_t)atomicAdd((unsigned long long*)&st->U, (unsigned long long)sz);
        k1 = k0 + sz;
      }
      D.kchunk[2 * w] = k0 + c;
      D.kchunk[2 * w + 1] = k1;
      S.bk = k0;
    }
  }
  int4* tm = D.TM + (int64_t)w * MTM;
  for (int32_t i = t; i < a; i += ABLOCK) tm[i] = S.tm[i];
  // the new pairs grouped by the appending workgroup that takes them (the hash bucket of the
  // key, mid_bucket): bucket k's run is [bcnt[k], bcnt[k + 1]) of the segment, so an appender
  // reads its own runs only (round 3: every appender read every new pair, ~16 MB a launch at
  // 30 k occurrences, and the appenders set the launch's length above ~10 k occurrences)
  int2* th = mid_th(D, par) + (int64_t)w * MTH;
  if (t <= MID_APP) S.bcnt[t] = 0;
  __syncthreads();
  int32_t k0 = 0, k1 = 0, r0 = -1, r1 = -1;
  if (t < b) {
    k0 = (int32_t)mid_bucket(max(S.th[t].y, 0), MID_APP);
    r0 = atomicAdd(&S.bcnt[k0], 1);
  }
  if (t + ABLOCK < b) {
    k1 = (int32_t)mid_bucket(max(S.th[t + ABLOCK].y, 0), MID_APP);
    r1 = atomicAdd(&S.bcnt[k1], 1);
  }
  __syncthreads();
  if (t == 0) {
    int32_t run = 0;
    for (int k = 0; k < MID_APP; k++) {
      const int32_t n = S.bcnt[k];
      S.bcnt[k] = run;
      run += n;
    }
    S.bcnt[MID_APP] = run;
  }
  __syncthreads();
  if (t <= MID_APP) D.mbk[((int64_t)par * NBA_MAX + w) * (MID_APP + 1) + t] = S.bcnt[t];
  if (r0 >= 0) th[S.bcnt[k0] + r0] = S.th[t];
  if (r1 >= 0) th[S.bcnt[k1] + r1] = S.th[t + ABLOCK];
  if (c) {
    __syncthreads();
    for (int32_t i = t; i < c; i += ABLOCK) klist_put(D, S.bk + i, S.kl[i]);
  }
}

// multi-rank (D.xrec set, the pipelined exchange): count changes go out as delta records
// (the producer applies its own with the hot-list check, the other ranks' imports probe by
// content); the record carries this rank's key id (pad = id + 1: the producer's own add).  Records are
// reserved per workgroup phase (mid_reserve) where the count is known, one wave at a time
// only on the rare paths (a run's later occurrences, a full LDS table).
__device__ inline unsigned long long* mid_xcnt(const Dev& D) {
  return (unsigned long long*)(D.xcnt ? D.xcnt : &D.st->ntouched);
}
__device__ inline void mid_put(const Dev& D, int64_t j, u64 h1, u64 h2, int32_t len, int32_t idL, int32_t g,
                               int32_t idR, int32_t delta, int32_t d) {
  DeltaRec r;
  r.h1 = h1;
  r.h2 = h2;
  r.len = len;
  r.idL = idL;
  r.g = g;
  r.idR = idR;
  r.delta = delta;
  r.pad = d + 1;
  x_put_rec(D, j, r, -72);
}
__device__ inline void mid_put_id(const Dev& D, int64_t j, int32_t d, int32_t delta) {
  mid_put(D, j, D.kh1[d], D.kh2[d], D.klen[d], D.krep[3 * (int64_t)d], D.krep[3 * (int64_t)d + 1],
          D.krep[3 * (int64_t)d + 2], delta, d);
}
__device__ inline void mid_emit(const Dev& D, u64 h1, u64 h2, int32_t len, int32_t idL, int32_t g, int32_t idR,
                                int32_t delta, int32_t d) {
  const u64 m = __ballot(1);
  const int lane = wave_lane();
  const int leader = __ffsll((long long)m) - 1;
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd(mid_xcnt(D), (unsigned long long)__popcll(m));
  base = __shfl(base, leader, 64);
  mid_put(D, (int64_t)base + __popcll(m & ((1ULL << lane) - 1)), h1, h2, len, idL, g, idR, delta, d);
}
__device__ inline void mid_emit_id(const Dev& D, int32_t d, int32_t delta) {
  mid_emit(D, D.kh1[d], D.kh2[d], D.klen[d], D.krep[3 * (int64_t)d], D.krep[3 * (int64_t)d + 1],
           D.krep[3 * (int64_t)d + 2], delta, d);
}
// n records of this workgroup (block-uniform call; n from LDS): the base index, one atomic
__device__ inline int64_t mid_reserve(const Dev& D, int64_t* s_base, int32_t n) {
  __syncthreads();
  if (threadIdx.x == 0) *s_base = n > 0 ? (int64_t)atomicAdd(mid_xcnt(D), (unsigned long long)n) : 0;
  __syncthreads();
  return *s_base;
}
// -v on key d: a count atomic, or a record (multi-rank; X: the exchange's instantiation of the
// kernel -- the one-rank kernels carry none of the record code)
template <bool X>
__device__ inline void mid_dec(const Dev& D, int32_t d, int32_t v) {
  if (X && D.xrec)
    mid_emit_id(D, d, v);
  else
    atomicAdd(&D.count[d], v);
}

// -1 on key d for a destroyed pair, staged in LDS.  One rank: not on W itself -- every pair
// of W is merged or destroyed by the merge, so the find sets count[W] = 0 once instead of
// every workgroup decrementing it
template <bool X>
__device__ inline void mid_dec_agg(const Dev& D, MidFindLds& S, const MidCtx& F, int32_t d) {
  if (!(X && D.xrec) && d == F.W) return;
  if (!agg_stage(S.agg, d, -1)) mid_dec<X>(D, d, -1);
}

// find-or-claim with the CAS as the first probe (an empty first slot is claimed, the key
// itself is found, anything else probes on)
__device__ inline int32_t mid_resolve(const Dev& D, u64 h1, u64 h2, int32_t len, bool* claimed) {
  const u64 k = probe_key(h1, h2, len);
  const u64 s0 = ht_first_slot(D, k);
  const u64 old = atomicCAS((unsigned long long*)&D.ht_key[s0], 0ULL, (unsigned long long)k);
  *claimed = old == 0;
  if (old == 0 || old == k) return (int32_t)s0;
  const u64 s1 = (s0 + 1) & ((u64)D.HC - 1);
  return ht_resolve(D, k, s1, ht_probe(D, s1), claimed);
}

// a new pair resolved on its own (a run's later occurrence, or the round's table is full)
template <bool X>
__device__ void mid_single(const Dev& D, MidFindLds& S, const MidCtx& F, u64 h1, u64 h2, int32_t len, int32_t idL,
                           int32_t g, int32_t idR, int32_t target) {
  bool claimed;
  const int32_t d = mid_resolve(D, h1, h2, len, &claimed);
  if (d < 0) return;
  if (claimed) {
    claim_payload(D, d, h1, h2, len, idL, g, idR);
    mid_claimed(D, S, d);
  } else {
    emit_check(D, &S.chk, d, len, h1, h2);
  }
  if (X && D.xrec)
    mid_emit(D, h1, h2, len, idL, g, idR, 1, d);
  else
    count_add_hot(D, S.hot, d, 1, F.th);
  mid_pair(D, S, F, target, d);
}

struct MidHalf {
  u64 pkey, h1, h2;
  int32_t len, idL, g, idR, target;
};

__device__ inline void mid_right(const Dev& D, const MidCtx& F, int32_t t, int32_t glR, bool cL, int32_t idc,
                                 int32_t lc, u64 c1, u64 c2, MidHalf& h) {
  const int32_t rl = cL ? F.wl : lc;
  const u64 r1 = cL ? F.w1 : c1, r2 = cL ? F.w2 : c2;
  const int64_t ny = 2 * (int64_t)rl - 1;
  combine_pw(F.w1, F.w2, glR, r1, r2, D.pw1[ny + 1], D.pw1[ny], D.pw2[ny + 1], D.pw2[ny], h.h1, h.h2);
  h.len = F.wl + rl;
  h.pkey = probe_key(h.h1, h.h2, h.len);
  h.idL = F.nid;
  h.g = glR;
  h.idR = cL ? F.nid : idc;
  h.target = t;
}

// the walk of merge.h find_walk: the first occurrence's new pairs are returned (grouped
// by the caller), a run's later occurrences resolve theirs on their own
template <bool X>
__device__ void mid_walk(const Dev& D, MidFindLds& S, const MidCtx& F, int32_t g, MidHalf& hl, bool& vl, MidHalf& hr,
                         bool& vr) {
  vl = vr = false;
  const int32_t W = F.W;
  const int4 tg = D.tok[g];
  if (tg.w != W) return;  // (a stale list entry)
  const int32_t p = tg.z;
  const int32_t b = g + tok_len(tg.y);
  const int4 tp = D.tok[p >= 0 ? p : g];
  const int4 tb = D.tok[b];
  if (p >= 0 && tp.w == W) return;  // not a run start
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
  mid_occ(D, S, F, g, F.wl | (tb.y & (int32_t)0xFFFF0000), b, c);
  if (pkb >= 0) mid_dec_agg<X>(D, S, F, pkb);
  if (pN) {
    mid_dec_agg<X>(D, S, F, tp.w);
    combine_pw(l1, l2, glL, F.w1, F.w2, F.pa1, F.pb1, F.pa2, F.pb2, hl.h1, hl.h2);
    hl.len = tok_len(tp.y) + F.wl;
    hl.pkey = probe_key(hl.h1, hl.h2, hl.len);
    hl.idL = tp.x;
    hl.g = glL;
    hl.idR = F.nid;
    hl.target = p;
    vl = true;
  }
  if (c >= 0) {
    mid_right(D, F, g, glR, cL, tc.x, tok_len(tc.y), c1, c2, hr);
    vr = true;
  }
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
    mid_occ(D, S, F, t, F.wl | (tb2.y & (int32_t)0xFFFF0000), b2, c2i);
    if (pkb2 >= 0) mid_dec_agg<X>(D, S, F, pkb2);
    if (c2i >= 0) {
      MidHalf h;
      mid_right(D, F, t, glR2, cL2, tc2.x, tok_len(tc2.y), d1, d2, h);
      mid_single<X>(D, S, F, h.h1, h.h2, h.len, h.idL, h.g, h.idR, h.target);
    }
    cur_c = c2i;
    cur_pkb = pkb2;
    cur_cL = cL2;
    lcur_c = tok_len(tc2.y);
  }
}

// round table slot of a new key; -1 when the probes run out (*ins: this thread inserted it)
__device__ inline int32_t mkc_slot(MidFindLds& S, const MidHalf& h, bool* ins) {
  int32_t s = (int32_t)((h.pkey * 0x9E3779B97F4A7C15ULL) >> (64 - 10)) & (MKC - 1);
  *ins = false;
#pragma unroll 1
  for (int probe = 0; probe < 16; probe++, s = (s + 1) & (MKC - 1)) {
    u64 c = S.key[s];
    if (c == 0) {
      c = atomicCAS((unsigned long long*)&S.key[s], 0ULL, (unsigned long long)h.pkey);
      if (c == 0) {
        *ins = true;
        return s;
      }
    }
    if (c == h.pkey) return s;
  }
  return -1;
}

// _tokens[n] = json.loads(key) (the new token's content in vsym) and the state the next select
// reads -- by appending workgroup 0 (it starts with nothing to wait for; on find workgroup 0
// these two dependent round trips delayed that workgroup's walk, the launch's last to end)
__device__ inline void mid_new_token(const Dev& D, const Sel& sel) {
  State* st = D.st;
  const int32_t t = threadIdx.x;
  const int32_t L = sel.widL, g = sel.wg, Rr = sel.widR;
  const int64_t vL = D.voff[L], vR = D.voff[Rr];
  const int64_t nL = D.voff[L + 1] - vL, nR = D.voff[Rr + 1] - vR;
  const int64_t pos = D.voff[sel.nid], ln = nL + 1 + nR;
  if (pos + ln > D.VSC) {
    if (t == 0) set_error(D, GEOBPE_ECAPACITY, -9);
  } else {
    for (int64_t i = t; i < ln; i += ABLOCK)
      D.vsym[pos + i] = i < nL ? D.vsym[vL + i] : (i == nL ? g : D.vsym[vR + i - nL - 1]);
    if (t == 0) D.voff[sel.nid + 1] = pos + ln;
  }
  if (t == 0) {
    st->iter = sel.iter + 1;
    st->K = sel.nid + 1;
    st->maxc = sel.maxc;
    st->ncand = sel.ncand;
  }
}

// what a find workgroup reads that depends on neither the Sel record nor each other, loaded
// in the launch's first round beside the Sel record (both parities' segment counts: the
// previous merge's parity is itself one of these loads)
struct MidPre {  // (scalars: an indexed pair would be a private array, which the compiler puts in LDS)
  int32_t pp, theta, seg0, seg1;
  int64_t spill0, spill1;
  int64_t kc0, kc1;  // this workgroup's klist chunk (its claims' list positions, mid_flush_lists)
};
__device__ inline MidPre mid_pre(const Dev& D, int32_t w) {
  MidPre m;
  const State* st = D.st;
  m.pp = st->place_par_prev;
  m.theta = st->theta;
  m.seg0 = D.mcnt[w].y;
  m.seg1 = D.mcnt[NBA_MAX + w].y;
  m.spill0 = st->mid_nh[0];
  m.spill1 = st->mid_nh[1];
  m.kc0 = D.kchunk[2 * w];
  m.kc1 = D.kchunk[2 * w + 1];
  return m;
}

// find workgroup w of G (merge parity par, decision sel)
template <bool X>
__device__ __attribute__((always_inline)) inline void mid_find_body(const Dev& D, const Sel& sel, int par, int32_t w,
                                                                    int32_t G, MidFindLds& S, const MidPre& M) {
  State* st = D.st;
  const int32_t t = threadIdx.x;
  dbg_stamp(D, 10);
  if (w == 0 && t == 0) {
    st->place_par = sel.decision == SEL_MERGE ? par : -1;
    if (sel.decision == SEL_DONE) {
      st->done = 1;
      st->maxc = 0;
    } else if (sel.decision == SEL_SKIP) {
      st->nskip += 1;
    }
  }
  if (sel.decision == SEL_DONE || sel.decision == SEL_STALL || sel.decision == SEL_IDLE) return;
  if (sel.decision == SEL_SKIP) {
    if (t == 0) D.chkcnt[w] = 0;
    if (sel.skip & SKIP_MEASURE) measure_max(D, w, G);
    if (sel.skip & SKIP_HOT) rebuild_hot_list(D, sel.theta_new, sel.build, w, G);
    return;
  }
  MidCtx F;
  F.W = sel.W;
  F.nid = sel.nid;
  F.wl = sel.wl;
  F.w1 = sel.w1;
  F.w2 = sel.w2;
  F.th = M.theta;
  F.par = par;
  F.iter = sel.iter;
  F.maxc = sel.maxc;
  {
    const int64_t nw = 2 * (int64_t)max(F.wl, 1) - 1;
    F.pa1 = D.pw1[nw + 1];
    F.pb1 = D.pw1[nw];
    F.pa2 = D.pw2[nw + 1];
    F.pb2 = D.pw2[nw];
  }
  // candidates: share w of the winner's list, then the previous merge's new pairs of key W
  // (find workgroup w's segment of them, and share w of the spill list)
  const int32_t nW = sel.kpn;
  const int32_t pp = M.pp;  // the previous merge's parity (-1: its pairs are in the lists)
  const int2* thp = mid_th(D, pp >= 0 ? pp : 0);
  const int64_t l0 = (int64_t)nW * w / G, nl = (int64_t)nW * (w + 1) / G - l0;
  const int64_t offW = sel.kpoff + l0;
  const int64_t nsg = pp >= 0 ? min((pp & 1) ? M.seg1 : M.seg0, MTH) : 0;
  const int64_t nsp = pp >= 0 ? min((pp & 1) ? M.spill1 : M.spill0, D.THcap - MSEG_TH) : 0;
  const int64_t s0 = nsp * w / G, ns = nsp * (w + 1) / G - s0;
  const int2* segp = thp + (int64_t)w * MTH;
  const int2* spp = thp + MSEG_TH + s0;
  const int64_t ncand = nl + nsg + ns;
  // (round 0's list candidate of this thread, loaded beside the hash powers: both depend only
  // on the Sel record, and the barrier below waits for every outstanding load anyway)
  const int32_t g0 = t < nl ? D.kpool[offW + t] : -1;
  for (int i = t; i < MKC; i += ABLOCK) {
    S.key[i] = 0;
    S.cnt[i] = 0;
  }
  for (int i = t; i < AggT<11>::N; i += ABLOCK) {
    S.agg.key[i] = -1;
    S.agg.val[i] = 0;
  }
  if (t == 0) {
    S.nocc = S.nm = S.chk = 0;
    S.ntm = S.nth = S.nkl = 0;
    S.hot.n = 0;
  }
  __syncthreads();
  dbg_stamp(D, 11);
  int64_t xdec_base = -1;  // (X: the decrement records' base, reserved with the last round's)
  int32_t xdec_ex = 0;
  for (int64_t c0 = 0; c0 < ncand; c0 += ABLOCK) {  // block-uniform rounds, one candidate per thread
    const int64_t i = c0 + t;
    MidHalf hl, hr;
    bool vl = false, vr = false;
    if (i < ncand) {
      int32_t g = -1;
      if (i < nl) {
        g = c0 == 0 ? g0 : D.kpool[offW + i];
      } else {
        const int2 e = i < nl + nsg ? segp[i - nl] : spp[i - nl - nsg];
        if (e.y == F.W) g = e.x;
      }
      if (g >= 0 && g < D.R) mid_walk<X>(D, S, F, g, hl, vl, hr, vr);  // (a bad list entry: no out-of-range read)
    }
    if (c0 == 0) dbg_stamp(D, 15);
    // ---- this round's new keys: LDS dedupe, then one resolve + count update per key
    bool il = false, ir = false;
    int32_t sl = -1, sr = -1;
    if (vl) {
      sl = mkc_slot(S, hl, &il);
      if (sl >= 0) atomicAdd(&S.cnt[sl], 1);
    }
    if (vr) {
      sr = mkc_slot(S, hr, &ir);
      if (sr >= 0) atomicAdd(&S.cnt[sr], 1);
    }
    if (il) {
      S.h1[sl] = hl.h1;
      S.h2[sl] = hl.h2;
      S.rep[sl] = make_int4(hl.len, hl.idL, hl.g, hl.idR);
      S.occ[atomicAdd(&S.nocc, 1)] = sl;
    }
    if (ir) {
      S.h1[sr] = hr.h1;
      S.h2[sr] = hr.h2;
      S.rep[sr] = make_int4(hr.len, hr.idL, hr.g, hr.idR);
      S.occ[atomicAdd(&S.nocc, 1)] = sr;
    }
    if (vl && sl < 0) mid_single<X>(D, S, F, hl.h1, hl.h2, hl.len, hl.idL, hl.g, hl.idR, hl.target);
    if (vr && sr < 0) mid_single<X>(D, S, F, hr.h1, hr.h2, hr.len, hr.idL, hr.g, hr.idR, hr.target);
    __syncthreads();
    if (c0 == 0) dbg_stamp(D, 16);
    const int32_t nocc = S.nocc;
    int64_t xb = 0;  // (one record per slot)
    if constexpr (X) {
      if (D.xrec) {
        if (c0 + ABLOCK >= ncand) {  // the last round: the decrement records (every walk is done, so
          // the staging is final) and W's own record go in the same reservation -- no second
          // returning atomic at the launch's end
          constexpr int PER = AggT<11>::N / ABLOCK;
          int32_t n = 0;
#pragma unroll
          for (int u = 0; u < PER; u++) {
            const int i = t + u * ABLOCK;
            n += S.agg.key[i] >= 0 && S.agg.val[i] != 0;
          }
          const int32_t own = t == 0 && S.nm ? 1 : 0;
          int32_t tot;
          xdec_ex = block_excl_scan(n + own, &tot, S.red);
          xb = mid_reserve(D, &S.xbase, nocc + tot);
          xdec_base = xb + nocc;
        } else {
          xb = mid_reserve(D, &S.xbase, nocc);
        }
      }
    }
    for (int32_t q = t; q < nocc; q += ABLOCK) {
      const int32_t s = S.occ[q];
      const int4 rp = S.rep[s];
      bool claimed;
      const u64 h1 = S.h1[s], h2 = S.h2[s];
      // (round 5 A/Bs, DESIGN 3: the count add beside the CAS, or its hot-list check deferred
      // under the pair writes, were both slower)
      const int32_t d = mid_resolve(D, h1, h2, rp.x, &claimed);
      S.did[s] = d;
      if (d < 0) {
        if (X && D.xrec) mid_put(D, xb + q, h1, h2, rp.x, rp.y, rp.z, rp.w, 0, -1);  // (no-op record)
        continue;
      }
      if (claimed) {
        claim_payload(D, d, h1, h2, rp.x, rp.y, rp.z, rp.w);
        mid_claimed(D, S, d);
      } else {
        emit_check(D, &S.chk, d, rp.x, h1, h2);
      }
      if (X && D.xrec)
        mid_put(D, xb + q, h1, h2, rp.x, rp.y, rp.z, rp.w, S.cnt[s], d);
      else
        count_add_hot(D, S.hot, d, S.cnt[s], F.th);
    }
    // the last round's walks are done, so every decrement is staged: out now, one atomic per
    // key, in flight under the new pairs' grouping and the list flush (at the launch's end they
    // were the last memory operations to drain; issued before the resolves they queued ahead of
    // the resolves' atomics: merge 100 +2 us, profiles/r5_s6/)
    if (!(X && D.xrec) && c0 + ABLOCK >= ncand)
      for (int i = t; i < AggT<11>::N; i += ABLOCK) {
        const int32_t k = S.agg.key[i], v = S.agg.val[i];
        if (k >= 0 && v != 0) atomicAdd(&D.count[k], v);
      }
    __syncthreads();
    if (c0 == 0) dbg_stamp(D, 17);
    if (vl && sl >= 0) {
      if (S.h1[sl] != hl.h1) set_error(D, GEOBPE_EHASH, -13);  // same probe key, other content
      if (S.did[sl] >= 0) mid_pair(D, S, F, hl.target, S.did[sl]);
    }
    if (vr && sr >= 0) {
      if (S.h1[sr] != hr.h1) set_error(D, GEOBPE_EHASH, -13);
      if (S.did[sr] >= 0) mid_pair(D, S, F, hr.target, S.did[sr]);
    }
    __syncthreads();
    for (int32_t q = t; q < nocc; q += ABLOCK) {  // clear the round's slots
      const int32_t s = S.occ[q];
      S.key[s] = 0;
      S.cnt[s] = 0;
    }
    if (t == 0) S.nocc = 0;
    __syncthreads();
  }
  mid_flush_lists(D, S, F.par, w, M.kc0, M.kc1);
  dbg_stamp(D, 12);
  // ---- the decrements (one atomic per key), W's merged pairs, merge count, hot list
  if (X && D.xrec) {  // as records: the nonzero slots, compacted behind one reservation
    constexpr int PER = AggT<11>::N / ABLOCK;
    static_assert(AggT<11>::N % ABLOCK == 0, "agg slots per thread");
    int32_t n = 0;
#pragma unroll
    for (int u = 0; u < PER; u++) {
      const int i = t + u * ABLOCK;
      n += S.agg.key[i] >= 0 && S.agg.val[i] != 0;
    }
    const int32_t own = t == 0 && S.nm ? 1 : 0;
    int64_t j;
    if (xdec_base >= 0) {  // (reserved with the last round's records)
      j = xdec_base + xdec_ex;
    } else {  // (no round: no candidate)
      int32_t tot;
      const int32_t ex = block_excl_scan(n + own, &tot, S.red);
      j = mid_reserve(D, &S.xbase, tot) + ex;
    }
    if (own) mid_put_id(D, j++, F.W, -S.nm);
#pragma unroll
    for (int u = 0; u < PER; u++) {
      const int i = t + u * ABLOCK;
      const int32_t k = S.agg.key[i], v = S.agg.val[i];
      if (k >= 0 && v != 0) mid_put_id(D, j++, k, v);
    }
  } else {  // (the decrements went out with the last round)
    // (mid_dec_agg: every pair of W is gone)
    if (w == 0 && t == 0) atomicAdd(&D.count[F.W], -F.maxc);
  }
  // (the merge's merged total: the next place sums the workgroups' counts into the log)
  hot_flush(D, S.hot);  // (syncs the workgroup first)
  if (t == 0) D.chkcnt[w] = min(S.chk, (int32_t)D.RC);
  dbg_stamp(D, 13);
}

// ---------------------------------------------------------------------- appends

// the key's slot in the append table (insert: claim an empty one); -1: not there / full
__device__ inline int32_t mpk_slot(MidAppLds& S, int32_t d, bool insert, bool* ins) {
  int32_t s = (int32_t)(((uint32_t)d * 0x85EBCA6Bu) >> (32 - 11)) & (MPK - 1);
  *ins = false;
#pragma unroll 1
  for (int probe = 0; probe < 64; probe++, s = (s + 1) & (MPK - 1)) {
    int32_t c = S.key[s];
    if (c == -1) {
      if (!insert) return -1;
      c = atomicCAS(&S.key[s], -1, d);
      if (c == -1) {
        *ins = true;
        return s;
      }
    }
    if (c == d) return s;
  }
  return -1;
}

constexpr int MP_UNR = 8;  // new-pair list entries in flight per thread

// appending workgroup b of A: the posting entries of merge pp's new pairs (the find
// workgroups' segments of TH(pp) and its spill list) whose key is in bucket b, except key
// `skip` -- one pass counts them per key (and keeps each entry with its rank in LDS), the
// lists grow where needed (one pool reservation per round), then the kept entries are
// written (a second pass over the new pairs only when more than MAE were kept).  Threads
// split the segments TPS to a segment; every thread strides the spill list.
// one new pair of merge pp in an appender: PASS 0 keeps it in LDS when its key is this
// appender's (compacted, one LDS reservation per wave instruction); PASS 1 / 2 are the
// fallback when more than MAE are kept -- 1 counts it for its key, 2 writes it
template <int PASS>
__device__ __attribute__((always_inline)) inline void mid_app_one(const Dev& D, MidAppLds& S, int2 h, int32_t skip,
                                                                  int32_t b, int32_t A) {
  const int32_t d = h.y;
  if (d < 0 || d == skip || mid_bucket(d, A) != (uint32_t)b) return;
  bool ins;
  if constexpr (PASS == 0) {
    const int32_t e = lds_reserve(&S.nent);
    if (e < MAE) S.ent[e] = h;
  } else if constexpr (PASS == 1) {
    const int32_t s = mpk_slot(S, d, true, &ins);
    if (s < 0) {
      S.full = 1;  // (more keys than the table: the lists are rebuilt)
      return;
    }
    atomicAdd(&S.cnt[s], 1);
    if (ins) S.occ[atomicAdd(&S.nocc, 1)] = s;
  } else {
    const int32_t s = mpk_slot(S, d, false, &ins);
    if (s < 0 || S.off[s] < 0) return;
    const int32_t r = atomicAdd(&S.cur[s], 1);
    D.kpool[(int64_t)S.off[s] + S.base[s] + r] = h.x;
  }
}
// every new pair of merge pp through mid_app_one: a wave takes whole segments of the find
// workgroups (64 lanes on consecutive entries, MP_UNR segments in flight; S.pre holds the
// segment counts), every thread strides the spill list
template <int PASS>
__device__ __attribute__((always_inline)) inline void mid_app_pass(const Dev& D, MidAppLds& S, int32_t pp,
                                                                   int32_t skip, int32_t b, int32_t A) {
  const int2* th = mid_th(D, pp);
  const int32_t NS = mid_G(D), t = threadIdx.x;
  const int32_t tot = S.pre[NS];  // (this bucket's runs of every segment, flattened)
  for (int32_t q0 = t; q0 < tot; q0 += MP_UNR * ABLOCK) {
    int2 h[MP_UNR];
#pragma unroll
    for (int u = 0; u < MP_UNR; u++) {
      const int32_t q = q0 + u * ABLOCK;
      if (q < tot) {
        const int32_t w = seg_of(S.pre, NS, q);
        h[u] = th[(int64_t)w * MTH + S.rb[w] + (q - S.pre[w])];
      } else {
        h[u] = make_int2(-1, -1);
      }
    }
#pragma unroll
    for (int u = 0; u < MP_UNR; u++) mid_app_one<PASS>(D, S, h[u], skip, b, A);
  }
  const int64_t nsp = min(D.st->mid_nh[pp], D.THcap - MSEG_TH);
  const int2* sp = th + MSEG_TH;
  for (int64_t i0 = t; i0 < nsp; i0 += MP_UNR * ABLOCK) {
    int2 h[MP_UNR];
#pragma unroll
    for (int u = 0; u < MP_UNR; u++) h[u] = i0 + u * ABLOCK < nsp ? sp[i0 + u * ABLOCK] : make_int2(-1, -1);
#pragma unroll
    for (int u = 0; u < MP_UNR; u++) mid_app_one<PASS>(D, S, h[u], skip, b, A);
  }
}

__device__ __attribute__((always_inline)) inline void mid_append_body(const Dev& D, int32_t pp, int32_t skip, int32_t b, int32_t A, MidAppLds& S) {
  State* st = D.st;
  const int32_t t = threadIdx.x;
  dbg_stamp(D, 30);
  if (A != MID_APP) {  // (the segments' runs are by MID_APP buckets: any other split rebuilds the lists)
    if (t == 0) st->kp_valid = 0;
    return;
  }
  for (int i = t; i < MPK; i += ABLOCK) {
    S.key[i] = -1;
    S.cnt[i] = 0;
    S.cur[i] = 0;
  }
  if (t == 0) S.nocc = S.nbig = S.full = S.nent = 0;
  {  // this bucket's run in every find workgroup's TH segment (mid_flush_lists grouped them)
    const int32_t NS = mid_G(D);
    int32_t len = 0;
    if (t < NS && b <= MID_APP - 1) {
      const int32_t cnt = min(D.mcnt[pp * NBA_MAX + t].y, MTH);
      const int32_t* bo = D.mbk + ((int64_t)pp * NBA_MAX + t) * (MID_APP + 1);
      const int32_t o0 = min(max(bo[b], 0), cnt), o1 = min(max(bo[b + 1], o0), cnt);
      S.rb[t] = o0;
      len = o1 - o0;
    }
    int32_t tot;
    const int32_t ex = block_excl_scan(len, &tot, S.red);
    if (t < NS) S.pre[t] = ex;
    if (t == 0) S.pre[NS] = tot;
  }
  __syncthreads();
  // ---- pass 1: this bucket's new pairs compacted into LDS, then counted per key (dense)
  mid_app_pass<0>(D, S, pp, skip, b, A);
  __syncthreads();
  const bool kept = S.nent <= MAE;
  if (kept) {
    const int32_t ne = S.nent;
    for (int32_t e = t; e < ne; e += ABLOCK) {
      const int2 h = S.ent[e];
      bool ins;
      const int32_t s = mpk_slot(S, h.y, true, &ins);
      if (s < 0) {
        S.full = 1;  // (more keys than the table: the lists are rebuilt)
        S.ent[e].x = -1;  // (dropped: the slot field marks it -- the packed word uses all 32 bits)
        continue;
      }
      const int32_t r = atomicAdd(&S.cnt[s], 1);
      if (ins) S.occ[atomicAdd(&S.nocc, 1)] = s;
      if (r < (1 << 21)) {
        S.ent[e].y = (int32_t)(((uint32_t)s << 21) | (uint32_t)r);
      } else {
        S.ent[e].x = -1;
        S.full = 1;
      }
    }
  } else {
    mid_app_pass<1>(D, S, pp, skip, b, A);
  }
  __syncthreads();
  dbg_stamp(D, 32);
  // ---- room for every key's new entries (a full list grows to 2x): one reservation per round
  const int32_t nocc = S.nocc;
  for (int32_t q0 = 0; q0 < nocc; q0 += ABLOCK) {  // block-uniform
    const int32_t q = q0 + t;
    int32_t sl = -1, d = -1, add = 0, n = 0, cap = 0, ncap = 0;
    if (q < nocc) {
      sl = S.occ[q];
      d = S.key[sl];
      add = S.cnt[sl];
      n = D.kp_n[d];
      cap = D.kp_cap[d];
      if (n + add > cap) ncap = max(2 * (n + add), 16);
    }
    int32_t tot;
    const int32_t ex = block_excl_scan(ncap, &tot, S.red);
    if (t == 0) S.pbase = tot ? (int64_t)atomicAdd((unsigned long long*)&st->kpool_used, (unsigned long long)tot) : 0;
    __syncthreads();
    if (q < nocc) {
      S.base[sl] = n;
      int32_t off = D.kp_off[d];
      if (ncap > 0 && S.pbase + ex + ncap > D.KPOOL) {  // no room: the lists are rebuilt, this
        S.full = 1;                                       // key's entries are not written
        off = -1;
      } else if (ncap > 0) {
        const int64_t at = S.pbase + ex;
        if (n <= TAIL_SMALL) {
          for (int32_t k = 0; k < n; k++) D.kpool[at + k] = D.kpool[(int64_t)off + k];
        } else {
          const int32_t x = atomicAdd(&S.nbig, 1);
          if (x < TAIL_BIG) {
            S.big_old[x] = off;
            S.big_new[x] = (int32_t)at;
            S.big_pre[x] = n;
          } else {
            S.full = 1;
          }
        }
        off = (int32_t)at;
        D.kp_off[d] = off;
        D.kp_cap[d] = ncap;
      }
      S.off[sl] = off;
      if (off >= 0) D.kp_n[d] = n + add;
    }
    __syncthreads();
  }
  dbg_stamp(D, 33);
  const int32_t nb = min(S.nbig, TAIL_BIG);
  if (nb > 0) {  // the big lists' old entries, by the whole workgroup
    int32_t tc;
    const int32_t cx = block_excl_scan(t < nb ? S.big_pre[t] : 0, &tc, S.red);
    __syncthreads();
    if (t < nb) S.big_pre[t] = cx;
    if (t == 0) S.big_pre[nb] = tc;
    __syncthreads();
    for (int32_t q = t; q < tc; q += ABLOCK) {
      const int32_t r = seg_of(S.big_pre, nb, q);
      const int32_t k = q - S.big_pre[r];
      D.kpool[(int64_t)S.big_new[r] + k] = D.kpool[(int64_t)S.big_old[r] + k];
    }
  }
  // ---- the entries
  if (kept) {
    const int32_t ne = S.nent;
    for (int32_t e = t; e < ne; e += ABLOCK) {
      const int2 x = S.ent[e];
      if (x.x < 0) continue;
      const int32_t sl = (int32_t)((uint32_t)x.y >> 21), r = x.y & ((1 << 21) - 1);  // (11 + 21 bits: unsigned)
      if (S.off[sl] >= 0) D.kpool[(int64_t)S.off[sl] + S.base[sl] + r] = x.x;
    }
  } else {  // (more than the LDS kept: a second pass over the new pairs, ranks afresh)
    mid_app_pass<2>(D, S, pp, skip, b, A);
  }
  __syncthreads();
  dbg_stamp(D, 35);
  if (S.full && t == 0) st->kp_valid = 0;
}

// workgroups 0..G-1: the find of merge `par` (find = 0: none, a flush; par < 0: the
// pipelined exchange's device parity); workgroups G..: the posting entries of the previous
// merge (st->place_par_prev), skipping this merge's winner
template <bool X>
__device__ __attribute__((always_inline)) inline void mid_find_main(const Dev& D, int par, int G, int find) {
  __shared__ union {
    MidFindLds f;
    MidAppLds a;
  } U;
  State* st = D.st;
  const MidPre pre = (int)blockIdx.x < G ? mid_pre(D, blockIdx.x) : MidPre{};
  if (par < 0) {  // pipelined exchange: parity from the device's iteration count; no-op while stalled
    if (st->stall) return;
    par = st->dgen & 1;
  }
  Sel sel = D.sel[par];
  // lists that lost entries (an append ran out of table or pool space): no merge until the
  // host rebuilds them -- the select wrote only what the next select overwrites (Sel, the
  // log entry, the new token's hashes)
  const bool valid = st->kp_valid != 0;
  if (!find || !valid) sel.decision = SEL_STALL;
  if ((int)blockIdx.x < G) {
    mid_find_body<X>(D, sel, par, blockIdx.x, G, U.f, pre);
    return;
  }
  if ((int)blockIdx.x == G && sel.decision == SEL_MERGE) mid_new_token(D, sel);
  const int32_t pp = st->place_par_prev;
  if (pp < 0 || !valid) return;
  const int32_t skip = sel.decision == SEL_MERGE ? sel.W : -1;
  mid_append_body(D, pp, skip, blockIdx.x - G, gridDim.x - G, U.a);
}
// X: the pipelined exchange's instantiation (records, the peer exchange's arrival); the one-rank
// loop's carries none of that code (round 6's first form: +1.4 us a launch from its registers)
template <bool X>
__global__ __launch_bounds__(ABLOCK) void k_mid_find(Dev D, int par, int G, int find) {
  mid_find_main<X>(D, par, G, find);
  if constexpr (X) x_arrive(D);  // (the peer exchange: this launch's records are out, exchange.h)
}

// ---------------------------------------------------------------------- select + place
// token rewrites and pk of merge st->place_par, share b of P; the EHASH check of the keys
// find workgroup b found
__device__ void mid_place_body(const Dev& D, int32_t b, int32_t P) {
  State* st = D.st;
  const int32_t t = threadIdx.x;
  dbg_stamp(D, 36);
  // The loads go out in three rounds, each depending only on the one before: (1) the check's
  // record count and the merge's parity; (2) this thread's check record, the Sel record, the
  // segment counts; (3) the check key's hashes and this thread's first merged occurrence and
  // new pair.  (Round 3's version ran the EHASH check's three dependent rounds, a barrier and
  // then the place's own three: this launch's place workgroups set its length.)
  const bool chk = b < D.NBA;  // (then consumed: the next find writes region b afresh)
  const int32_t nchk = chk ? min(D.chkcnt[b], (int32_t)D.RC) : 0;
  const int32_t par = st->place_par;
  const NewPair* reg = D.chk + (int64_t)b * D.RC;
  NewPair c0;
  const bool hc = t < nchk;
  if (hc) c0 = reg[t];
  const int32_t G = mid_G(D);
  Sel sel;
  sel.decision = SEL_STALL;
  int4 mc = make_int4(0, 0, 0, 0);
  int64_t nms = 0, nhs = 0;
  int32_t v0 = 0;  // (workgroup 0: the find workgroups' merged counts, summed below)
  if (par >= 0) {
    sel = D.sel[par];
    if (b < G) mc = D.mcnt[par * NBA_MAX + b];
    nms = min(st->mid_nm[par], D.TMcap - MSEG_TM);
    nhs = min(st->mid_nh[par], D.THcap - MSEG_TH);
    if (b == 0 && t < G) v0 = D.mcnt[par * NBA_MAX + t].z;
  }
  const bool go = par >= 0 && sel.decision == SEL_MERGE;  // (block-uniform)
  // find workgroup b's segments (b < G), share b of the spill lists
  const int4* tms = D.TM + (int64_t)b * MTM;
  const int2* th = mid_th(D, par >= 0 ? par : 0);
  const int2* ths = th + (int64_t)b * MTH;
  int64_t m0 = 0, nm = 0, h0 = 0, nh = 0;
  const int32_t sm = min(mc.x, MTM), sh = min(mc.y, MTH);
  int4 e = make_int4(0, 0, 0, 0);
  int2 h = make_int2(0, 0);
  if (go) {
    m0 = nms * b / P;
    nm = sm + (nms * (b + 1) / P - m0);
    h0 = nhs * b / P;
    nh = sh + (nhs * (b + 1) / P - h0);
    if (t < nm) e = t < sm ? tms[t] : D.TM[MSEG_TM + m0 + t - sm];
    if (t < nh) h = t < sh ? ths[t] : th[MSEG_TH + h0 + t - sh];
  }
  u64 kh1 = 0, kh2 = 0;
  int32_t kln = 0;
  if (hc) {
    kh1 = D.kh1[c0.target];
    kh2 = D.kh2[c0.target];
    kln = D.klen[c0.target];
  }
  const int32_t nid = sel.nid;
  auto place_tm = [&](const int4& x) {  // a merged occurrence's token rewrites
    *reinterpret_cast<int2*>(D.tok + x.x) = make_int2(nid, x.y);
    D.tok[x.z] = make_int4(-1, 0, -1, -1);
    if (x.w >= 0)
      *tok_f(D, x.w, 2) = x.x;
    else
      *tok_f(D, x.x, 3) = -1;
  };
  if (t < nm) place_tm(e);
  if (t < nh) *tok_f(D, h.x, 3) = h.y;
  if (hc && (kh1 != c0.h1 || kh2 != c0.h2 || kln != c0.len)) set_error(D, GEOBPE_EHASH, t);
  for (int64_t i = t + ABLOCK; i < nm; i += ABLOCK) place_tm(i < sm ? tms[i] : D.TM[MSEG_TM + m0 + i - sm]);
  for (int64_t i = t + ABLOCK; i < nh; i += ABLOCK) {
    const int2 x = i < sh ? ths[i] : th[MSEG_TH + h0 + i - sh];
    *tok_f(D, x.x, 3) = x.y;
  }
  for (int32_t i = t + ABLOCK; i < nchk; i += ABLOCK) {
    const NewPair x = reg[i];
    const int32_t d = x.target;
    if (!key_is(D, d, x.h1, x.h2, x.len)) set_error(D, GEOBPE_EHASH, i);
  }
  if (chk) {
    __syncthreads();  // (every thread has read the count)
    if (t == 0) D.chkcnt[b] = 0;
  }
  if (go && b == 0) {  // the merge's merged occurrences: the find workgroups' counts, summed
    int32_t v = v0;
    for (int32_t i = t + ABLOCK; i < G; i += ABLOCK) v += D.mcnt[par * NBA_MAX + i].z;
    __shared__ int32_t s_red[ABLOCK / 64];
    int32_t tot;
    block_excl_scan(v, &tot, s_red);
    if (t == 0) D.log[sel.iter].nmerged = tot;
  }
  dbg_stamp(D, 37);
}

// workgroup 0: select (par >= 0; INT32_MIN: place only); workgroups 1..P: the token
// rewrites of merge st->place_par.  Workgroup 0 records which merge's new pairs the next
// find's appends take (place_par_prev) and resets its parity's list cursors (nothing else
// in this launch reads them).
// (nimp > 0: the peer exchange's import of the previous launch's records first, in workgroups
// 1..nimp, which the select waits for; exchange.h)
__global__ __launch_bounds__(ABLOCK) void k_mid_sel(Dev D, int par, int run_end, int nimp) {
  if (blockIdx.x > 0) {
    if ((int)blockIdx.x - 1 < nimp) {
      __shared__ XImpLds X;
      x_import_share(D, X, blockIdx.x - 1, nimp, false);
    }
    mid_place_body(D, blockIdx.x - 1, gridDim.x - 1);
    return;
  }
  __shared__ int32_t s_red[SBLOCK / 64];
  __shared__ SelStage S;
  State* st = D.st;
  const bool xpend = nimp > 0 && st->xpend != 0;  // (read before any workgroup can change it)
  if (threadIdx.x == 0) st->place_par_prev = st->place_par;
  if (par == INT32_MIN) return;
  if (par < 0) {  // pipelined exchange: parity from the device's iteration count; no-op while stalled
    if (nimp > 0) {
      if (!x_import_wait(D, xpend, nimp)) return;
    } else if (st->stall) {
      return;
    }
    const int32_t g = st->dgen + 1;
    par = g & 1;
    __syncthreads();  // every thread has read dgen
    if (threadIdx.x == 0) st->dgen = g;
  }
  if (threadIdx.x == 0) {
    st->mid_nm[par] = 0;
    st->mid_nh[par] = 0;
  }
  if (!st->kp_valid) {  // the lists lost entries: no merge until the host rebuilds them
    if (threadIdx.x == 0) {
      Sel o{};
      o.decision = SEL_STALL;
      D.sel[par] = o;
    }
    return;
  }
  select_core<false>(D, par, S, s_red, nullptr, run_end);
}

// after a flush (k_mid_sel place-only + k_mid_find appends-only): nothing is pending
__global__ void k_mid_flushed(Dev D) {
  if (threadIdx.x == 0) {
    D.st->place_par = -1;
    D.st->place_par_prev = -1;
    D.st->mid_nh[0] = D.st->mid_nh[1] = 0;
    D.st->mid_nm[0] = D.st->mid_nm[1] = 0;
  }
}
