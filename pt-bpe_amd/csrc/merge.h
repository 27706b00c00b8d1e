// merge.h -- one merge of BPE.step (foldingdiff/bpe.py:1792-2166) after k_select has
// chosen the winner W: k_find and k_commit.  Included once, by kernels.h.
//
// The cost of a merge is global-memory round trips and global atomics.  A design
// where every workgroup resolves the new pair keys of its own occurrences sends
// each hot key to the key table once per workgroup (256 same-address CASes) and
// each count to memory once per (workgroup, key) -- in the heavy early merges that
// was 30 of k_apply's 56 us (profiles/r2_base/apply_timeline.txt).  Here every key
// has ONE owner workgroup, chosen from its content (the first key-table slot of its
// probe key): find workgroups group their occurrences' new keys and count
// decrements by owner, commit workgroups aggregate each owner's keys across all
// finders, resolve every key once and update every count once.
//
//  k_find   (NBA x 1024; read-only on the token state): the winner's candidate
//           slots from the posting index (region r's bucket of W + 1/NBA of the
//           log of W's owner), run starts, greedy walks, neighbour roles, the new
//           neighbour pairs' content hashes; per round an LDS dedupe of the new
//           keys, their occurrence slots grouped per key (T), one record per
//           (key, owner) and the LDS-aggregated count decrements per owner.
//  k_commit (NBA x 1024): the token rewrites of find region j; owner j's records
//           from every finder -> LDS dedupe -> one key-table resolve (claim or
//           find) per key -> pk of every occurrence slot, the owner's posting log,
//           one count update per key (+ hot-list crossing check).
// A posting index that is stale is rebuilt by k_find in the same iteration
// (rank-local, so ranks never disagree on what an iteration does).
#pragma once
// (included inside namespace gb)

// k_find's outputs (merge entries, key / decrement records, T slots) are read once, by
// k_commit / k_place on other XCDs.  Plain stores: non-temporal (round 2) and write-through
// (round 5: each scattered 4-16-B store then goes to memory, k_find 29.5 -> 41.3 us) stores
// were measured slower
template <typename V>
__device__ inline void out_store(V* p, const V& v) {
  *p = v;
}

// a load the compiler issues where it stands: a relaxed workgroup-scope atomic load (a plain
// global_load in the ISA), which it does not sink into the branch that uses the value -- a plain
// load only one path uses was moved there and waited for at once
__device__ inline int2 ld_now(const int2* p) {
  const unsigned long long v = __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
  return make_int2((int32_t)(v & 0xFFFFFFFFu), (int32_t)(v >> 32));
}
__device__ inline int32_t ld_now(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <typename T>
__device__ inline T ld_now_t(const T* p) {  // (any 8-B multiple, 8 B at a time)
  static_assert(sizeof(T) % 8 == 0, "8-B multiple");
  T r;
  const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
  unsigned long long* o = reinterpret_cast<unsigned long long*>(&r);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 8); i++)
    o[i] = __hip_atomic_load(q + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return r;
}
__device__ inline u64 ld_now(const u64* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ inline KRec ld_rec(const KRec* p) {  // (six 8-B loads)
  KRec r;
  const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
  unsigned long long* o = reinterpret_cast<unsigned long long*>(&r);
#pragma unroll
  for (int i = 0; i < 6; i++) o[i] = __hip_atomic_load(q + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return r;
}

// the record counts finder r sent owner o, finder-major, so a finder's end writes whole lines
// (owner-major, its 2 x NBA counts were NBA-strided 4-B writes: 2 x 65 536 partial lines a
// launch written back at k_find's end)
__device__ inline int64_t cnt_at(const Dev& D, int32_t o, int32_t r) { return (int64_t)r * D.NBA + o; }
// the two counts of a (finder, owner) as one int2 in cntK (allocated 2 x NBA^2), so an owner's
// first round loads one strided line set instead of two
__device__ inline int2 cnt_pair(const Dev& D, int32_t o, int32_t r) {
  return reinterpret_cast<const int2*>(D.cntK)[cnt_at(D, o, r)];
}

// chunked per-owner posting log: entry k of owner o
__device__ inline int64_t log_addr(const Dev& D, int o, int64_t k) {
  return (int64_t)D.pch[(int64_t)o * D.MAXCH + k / D.CHUNK] * D.CHUNK + k % D.CHUNK;
}
__device__ inline int64_t log_len(const Dev& D, int o) {
  const int32_t nc = D.pnch[o];
  return nc > 0 ? (int64_t)(nc - 1) * D.CHUNK + D.pfill[o] : 0;
}

// posting index of residue region r (one workgroup, hist: NBKT ints of LDS): counting
// sort of the region's live pairs by key bucket.  Entries of key W (>= 0) are also
// pushed to the candidate queue q (capacity FMQ; *qn counts all, the overflow is
// found again by the bucket read that follows).
__device__ void build_region_postings(const Dev& D, int32_t r, int32_t* hist, int32_t W, int32_t* q, int32_t* qn) {
  __shared__ int32_t s_red[ABLOCK / 64];
  constexpr int PER = NBKT / ABLOCK;
  const int64_t g0 = (int64_t)r * D.PR, g1 = min(D.R, g0 + D.PR);
  constexpr int UNR = 16;  // pk loads in flight per thread
  for (int i = threadIdx.x; i < NBKT; i += ABLOCK) hist[i] = 0;
  __syncthreads();
  for (int64_t g = g0 + threadIdx.x; g < g1; g += UNR * ABLOCK) {
    int32_t d[UNR];
#pragma unroll
    for (int u = 0; u < UNR; u++) d[u] = g + u * ABLOCK < g1 ? tok_pk(D, g + u * ABLOCK) : -1;
#pragma unroll
    for (int u = 0; u < UNR; u++)
      if (d[u] >= 0) atomicAdd(&hist[post_bkt(d[u])], 1);
  }
  __syncthreads();
  int32_t sum = 0;
  for (int k = 0; k < PER; k++) sum += hist[threadIdx.x * PER + k];
  int32_t tot;
  int32_t run = block_excl_scan(sum, &tot, s_red);
  int32_t* off = D.poff + (int64_t)r * (NBKT + 1);
  __syncthreads();
  for (int k = 0; k < PER; k++) {
    const int b = threadIdx.x * PER + k;
    const int32_t c = hist[b];
    hist[b] = run;
    off[b] = run;
    run += c;
  }
  if (threadIdx.x == 0) off[NBKT] = tot;
  __syncthreads();
  int2* out = D.post + (int64_t)r * D.PR;
  for (int64_t g = g0 + threadIdx.x; g < g1; g += UNR * ABLOCK) {
    int32_t d[UNR];
#pragma unroll
    for (int u = 0; u < UNR; u++) d[u] = g + u * ABLOCK < g1 ? tok_pk(D, g + u * ABLOCK) : -1;
#pragma unroll
    for (int u = 0; u < UNR; u++) {
      if (d[u] < 0) continue;
      const int32_t slot = (int32_t)(g + u * ABLOCK);
      out[atomicAdd(&hist[post_bkt(d[u])], 1)] = make_int2(d[u], slot);
      if (d[u] == W) {
        const int32_t j = atomicAdd(qn, 1);
        if (j < FMQ) q[j] = slot;
      }
    }
  }
  __syncthreads();
}

// record of a key found (not claimed): the next k_find checks it against the key's
// canonical hashes (EHASH)
__device__ inline void emit_check(const Dev& D, int32_t* s_np, int32_t d, int32_t len, u64 h1, u64 h2) {
  NewPair e;
  e.target = d;
  e.slot = -1;
  e.len = len;
  e.delta = 0;
  e.h1 = h1;
  e.h2 = h2;
  const int32_t j = atomicAdd(s_np, 1);
  if (j < D.RC)
    D.chk[(int64_t)blockIdx.x * D.RC + j] = e;
  else
    atomicAdd((unsigned long long*)&D.st->nunchecked, 1ULL);
}

// EHASH check of the keys the previous commit / import found (not claimed): their
// content hashes must be the key's canonical ones
__device__ inline void check_found(const Dev& D, int32_t r) {
  const int32_t n = D.chkcnt[r];
  const NewPair* reg = D.chk + (int64_t)r * D.RC;
  for (int32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const NewPair e = reg[i];
    const int32_t d = e.target;
    if (!key_is(D, d, e.h1, e.h2, e.len)) set_error(D, GEOBPE_EHASH, i);
  }
}

// ---------------------------------------------------------------------- k_find
// An (owner, finder) segment of KS is SK 48-B slots.  In the heavy merges a finder sends an owner
// ~1.5 key records and ~1.5 decrement records, so each segment's writes are a few bytes of one
// line: the first DSH decrement records therefore go into slot 0, in the line the key records
// (slots 1..SK-1) dirty anyway, and only the rest into DS.  (Separate DS segments wrote one more
// 64-B sector per segment: ~4 MB of k_find's ~16 MB written per heavy launch, all written back at
// the kernel boundary.)
// (The segment's record counts in slot 0 too, so that k_commit's first round found them in the
// line of its records, measured no faster: k_find's 256 more scattered stores cost what the
// commit saved, profiles/r6_ab/dsh/.)
constexpr int DSH = (int)(sizeof(KRec) / sizeof(int2));  // decrement records in slot 0
constexpr int SKR = SK - 1;                              // key records per segment
__device__ inline int64_t krec_at(int64_t seg, int32_t j) { return seg * SK + 1 + j; }
__device__ inline int2* dec_at(const Dev& D, int64_t seg, int32_t j) {
  return j < DSH ? reinterpret_cast<int2*>(D.KS + seg * SK) + j : D.DS + seg * SD + (j - DSH);
}
// k_commit -> k_place: a published record's {key id, posting-log position} overwrites its {g, idR}
// (read only by the commit's resolve, before the publish), so k_place's one 16-B load of the
// record's tail {id, log position, n, tstart} is one line (a separate id array was a second
// line per record, and one more dirty sector per segment at the commit's end)
static_assert(offsetof(KRec, g) == 32 && offsetof(KRec, idR) == 36 && offsetof(KRec, n) == 40 &&
                  offsetof(KRec, tstart) == 44, "a record's 16-B tail");
__device__ inline int2* rec_id(const Dev& D, int64_t at) { return reinterpret_cast<int2*>(&D.KS[at].g); }
__device__ inline int4 rec_tail(const Dev& D, int64_t at) { return ld_now_t(reinterpret_cast<const int4*>(&D.KS[at].g)); }

struct FHalf {  // a new neighbour pair of a merged occurrence
  u64 pkey, h1, h2;
  int32_t len, idL, g, idR, target;
};

struct FindCtx {
  int32_t W, nid, wl, ll, r, par;  // (ll: residues of W's left part)
  u64 w1, w2;
  u64 pa1, pb1, pa2, pb2;  // P^(2 wl), P^(2 wl - 1) of both bases (the left key's right part is W)
  bool to_delta;
};

// LDS of k_find (the posting rebuild's histogram shares the dedupe arrays)
struct FindLds {
  union {
    int32_t hist[NBKT];
    struct {
      u64 kkey[FKC];
      u64 kh1[FKC];
      int32_t kcnt[FKC];
      int32_t kst[FKC];
      int32_t kat[FKC];  // the key's record (KS index) this round: T entries carry it (k_place)
      AggT<12> agg;  // count decrements of this workgroup
    } m;
  } u;
  int32_t q[FMQ];
  int32_t curK[NBA_MAX], curD[NBA_MAX];
  int32_t red[ABLOCK / 64];
  int32_t qn, n, tb, fits, ktot;
  int32_t qsteal;  // the round's next unclaimed candidate (candidate stealing)
};

__device__ inline void emit_occ(const Dev& D, FindCtx& F, int32_t* s_n, int32_t a, int32_t ya, int32_t b, int32_t c) {
  LEntry e;
  e.a = a;
  e.ya = ya;
  e.b = b;
  e.c = c;
  // one LDS reservation per wave instruction (the active lanes are the callers)
  const u64 m = __ballot(1);
  const int lane = wave_lane();
  const int leader = __ffsll((long long)m) - 1;
  int32_t base = 0;
  if (lane == leader) base = atomicAdd(s_n, __popcll(m));
  base = __shfl(base, leader, 64);
  const int32_t j = base + __popcll(m & ((1ULL << lane) - 1));
  if (j < D.LC) {
    out_store(&D.L[(int64_t)F.r * D.LC + j], e);
  } else {
    const int64_t k = atomicAdd((unsigned long long*)&D.st->L_ovf2[F.par], 1ULL);
    if (k < D.Lovf_cap)
      D.Lovf[k] = e;
    else
      set_error(D, GEOBPE_ECAPACITY, -10);
  }
}

// a key record into its owner's slot of this finder (or the overflow list)
// (returns the record's index in KS -- the overflow list KO is KS's tail -- or -1)
__device__ inline int32_t emit_krec(const Dev& D, const FindCtx& F, int32_t* curK, const FHalf& h, int32_t n,
                                    int32_t tstart) {
  KRec k;
  k.pkey = h.pkey;
  k.h1 = h.h1;
  k.h2 = h.h2;
  k.len = h.len;
  k.idL = h.idL;
  k.g = h.g;
  k.idR = h.idR;
  k.n = n;
  k.tstart = tstart;
  const int o = owner_of_key(D, h.pkey);
  const int32_t j = atomicAdd(&curK[o], 1);
  if (j < SKR) {
    const int64_t at = krec_at((int64_t)o * D.NBA + F.r, j);
    out_store(&D.KS[at], k);
    return (int32_t)at;
  }
  const int64_t x = atomicAdd((unsigned long long*)&D.st->nko2[F.par], 1ULL);
  if (x < D.KO_cap) {
    D.KO[x] = k;
    return (int32_t)((int64_t)D.NBA * D.NBA * SK + x);
  }
  set_error(D, GEOBPE_ECAPACITY, -41);
  return -1;
}
__device__ inline void emit_single(const Dev& D, const FindCtx& F, int32_t* curK, const FHalf& h) {
  emit_krec(D, F, curK, h, 1, -(h.target + 1));
}

__device__ inline void dec_add(const Dev& D, const FindCtx& F, AggT<12>& agg, int32_t d, int32_t v) {
  if (!agg_stage(agg, d, v)) global_add(D, d, v, F.to_delta);
}

// the new key (X, glR, right) of occurrence t: right = X when c is a left part
__device__ inline void right_half(const Dev& D, const FindCtx& F, const FindLds& S, int32_t t, int32_t glR, bool cL,
                                  int32_t idc, int32_t lc, u64 c1, u64 c2, FHalf& h) {
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

// a candidate slot g of W: confirm it and, at a run start, walk the run greedily left
// to right (bpe.py:1888-1916): merge (t, b), skip (b, c), merge (c, d) if it is W
// too, ...  Neighbour roles without any write: c is a left part iff pk[c] == W; the
// run start's left neighbour p is a right part iff the W-run ending at (pp, p) has
// odd length.  The first occurrence's new keys are returned (grouped by the caller),
// a run's later occurrences send theirs as single records.
// (returns true when g is no occurrence to walk: a stale posting or not a run start)
__device__ bool find_walk(const Dev& D, FindCtx& F, FindLds& S, int32_t g, FHalf& hl, bool& vl, FHalf& hr,
                          bool& vr) {
  vl = vr = false;
  const int32_t W = F.W;
  // round 1: g, b and c together -- an occurrence of W is a left part at g and a right part at
  // b, b = g + len(L) for the winner's own split (L, R), and c = g + len(W) when b has a right
  // neighbour (whatever the split: the pair's length is the key's)
  const int32_t bs = min(g + F.ll, D.R - 1), cs = min(g + F.wl, D.R - 1);
  const int4 tg = D.tok[g];  // {tid, tlen, tprev, pk}
  int2 tb = make_int2(*tok_f(D, bs, 1), *tok_f(D, bs, 3));  // {.y, .w}: length word, pk
  const int4 tcs = make_int4(*tok_f(D, cs, 0), *tok_f(D, cs, 1), 0, *tok_f(D, cs, 3));
  if (tg.w != W) return true;
  int32_t b = bs;
  if (tok_len(tg.y) != F.ll) {  // another split of W's content (a key is its content, so (AB, C) and
    b = g + tok_len(tg.y);       // (A, BC) are one key): b from g's record, one more round here only
    tb = make_int2(*tok_f(D, b, 1), *tok_f(D, b, 3));
  }
  dbg_stamp(D, 40);
  const int32_t p = tg.z;
  // round 2: the run start's left context
  const int32_t ip = p >= 0 ? p : g;
  const int4 tp = D.tok[ip];
  if (p >= 0 && tp.w == W) return true;  // not a run start: its run's start walks it
  dbg_stamp(D, 41);
  const int32_t glL = p >= 0 ? next_glue(D, tp.y, g - 1) : 0;
  const int32_t glR = next_glue(D, tb.x, g + F.wl - 1);
  const int32_t pkb = tb.y;
  const int32_t c = pkb >= 0 ? cs : -1;
  const int4 tc = pkb >= 0 ? tcs : tg;
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
  dbg_stamp(D, 42);
  // the first occurrence (g, b)
  emit_occ(D, F, &S.n, g, F.wl | (tb.x & (int32_t)0xFFFF0000), b, c);
  if (pkb >= 0) dec_add(D, F, S.u.m.agg, pkb, -1);
  if (pN) {
    dec_add(D, F, S.u.m.agg, tp.w, -1);
    combine_pw(l1, l2, glL, F.w1, F.w2, F.pa1, F.pb1, F.pa2, F.pb2, hl.h1, hl.h2);
    hl.len = tok_len(tp.y) + F.wl;
    hl.pkey = probe_key(hl.h1, hl.h2, hl.len);
    hl.idL = tp.x;
    hl.g = glL;
    hl.idR = F.nid;
    hl.target = p;
    vl = true;
  }
  dbg_stamp(D, 43);
  if (c >= 0) {
    right_half(D, F, S, g, glR, cL, tc.x, tok_len(tc.y), c1, c2, hr);
    vr = true;
  }
  dbg_stamp(D, 44);
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
    emit_occ(D, F, &S.n, t, F.wl | (tb2.y & (int32_t)0xFFFF0000), b2, c2i);
    if (pkb2 >= 0) dec_add(D, F, S.u.m.agg, pkb2, -1);
    if (c2i >= 0) {
      FHalf h;
      right_half(D, F, S, t, glR2, cL2, tc2.x, tok_len(tc2.y), d1, d2, h);
      emit_single(D, F, S.curK, h);
    }
    cur_c = c2i;
    cur_pkb = pkb2;
    cur_cL = cL2;
    lcur_c = tok_len(tc2.y);
  }
  return false;
}

// LDS dedupe slot of a new key (*res: this thread inserted it); -1 when the probes
// run out (the half then goes as a single record)
__device__ inline int32_t fkc_find(FindLds& S, const Dev& D, u64 k, u64 h1, bool* res) {
  int32_t h = (int32_t)((k * 0x9E3779B97F4A7C15ULL) >> (64 - 11)) & (FKC - 1);
#pragma unroll 1
  for (int probe = 0; probe < 16; probe++, h = (h + 1) & (FKC - 1)) {
    u64 c = S.u.m.kkey[h];
    if (c == 0) {
      c = atomicCAS((unsigned long long*)&S.u.m.kkey[h], 0ULL, (unsigned long long)k);
      if (c == 0) {
        S.u.m.kh1[h] = h1;
        *res = true;
        return h;
      }
    }
    if (c == k) {
      *res = false;
      return h;
    }
  }
  *res = false;
  return -1;
}

// the round's dedupe slot (s), insert flag and rank within the slot of one new key per lane
// (round 5 A/B: lanes of a wave holding the same key sharing one probe and one counter add
// were slower, DESIGN 8 -- the same-key LDS atomics were not the cost)
__device__ inline void fkc_group(FindLds& S, const Dev& D, bool v, const FHalf& h, int32_t& s, bool& ins, int32_t& rank) {
  s = -1;
  ins = false;
  rank = 0;
  if (v) {
    s = fkc_find(S, D, h.pkey, h.h1, &ins);
    if (s >= 0) rank = atomicAdd(&S.u.m.kcnt[s], 1);
  }
}

__global__ __launch_bounds__(ABLOCK) void k_find(Dev D, int to_delta, int par) {
  __shared__ FindLds S;
  State* st = D.st;
  if (par < 0) {  // pipelined exchange (k_select set dgen)
    if (st->stall) return;
    par = st->dgen & 1;
  }
  const int32_t r = blockIdx.x;
  dbg_stamp(D, 10);
  const Sel sel = D.sel[par];
  check_found(D, r);
  if (sel.decision != SEL_MERGE) return;
  FindCtx F;
  F.W = sel.W;
  F.nid = sel.nid;
  F.wl = sel.wl;
  F.ll = D.vlen[sel.widL];
  F.r = r;
  F.par = par;
  F.w1 = sel.w1;
  F.w2 = sel.w2;
  F.to_delta = to_delta != 0;
  {
    const int64_t nw = 2 * (int64_t)max(F.wl, 1) - 1;
    F.pa1 = D.pw1[nw + 1];
    F.pb1 = D.pw1[nw];
    F.pa2 = D.pw2[nw + 1];
    F.pb2 = D.pw2[nw];
  }
  if (threadIdx.x == 0) {
    S.qn = 0;
    S.n = 0;
    S.tb = 0;
  }
  for (int i = threadIdx.x; i < NBA_MAX; i += ABLOCK) S.curK[i] = S.curD[i] = 0;
  // candidates: region r's bucket of W (+ 1/NBA of the log of W's owner)
  const int32_t W = F.W;
  const int o = sel.wown;
  int32_t lo = 0, n1 = 0;
  int64_t ls0 = 0, ls1 = 0;
  bool queued = false;  // the rebuild queued the bucket's W entries already
  if (sel.rebuild) {
    __syncthreads();
    build_region_postings(D, r, S.u.hist, W, S.q, &S.qn);
    if (threadIdx.x == 0) {
      D.pnch[r] = 0;  // (no finder reads a log in a rebuilding iteration)
      D.pfill[r] = 0;
      if (r == 0) {
        st->pool_used = 0;
        st->post_valid = 1;
        st->plog_ovf = 0;
        st->npost += 1;
      }
    }
    queued = S.qn <= FMQ;
  }
  if (W >= 0 && !queued) {
    {
      const int32_t* off = D.poff + (int64_t)r * (NBKT + 1);
      const uint32_t bk = post_bkt(W);
      lo = off[bk];
      n1 = off[bk + 1] - lo;
      if (!sel.rebuild) {
        const int64_t nlog = log_len(D, o);
        ls0 = nlog * r / D.NBA;
        ls1 = nlog * (r + 1) / D.NBA;
      }
    }
  }
  // dedupe + aggregation state
  for (int i = threadIdx.x; i < FKC; i += ABLOCK) {
    S.u.m.kkey[i] = 0;
    S.u.m.kcnt[i] = 0;
  }
  for (int i = threadIdx.x; i < AggT<12>::N; i += ABLOCK) {
    S.u.m.agg.key[i] = -1;
    S.u.m.agg.val[i] = 0;
  }
  __syncthreads();
  dbg_stamp(D, 11);
  const int64_t ntot = queued ? (int64_t)S.qn : n1 + (ls1 - ls0);
  const int2* P = D.post + (int64_t)r * D.PR + lo;
  dbg_val(D, 60, ntot + 1);  // (debug timeline: posting entries scanned, +1)
  int64_t dbg_nq = 0;
  for (int64_t c0 = 0; c0 < ntot; c0 += FMQ) {  // block-uniform
    int32_t nq;
    if (queued) {
      nq = (int32_t)ntot;
    } else {
      __syncthreads();
      if (threadIdx.x == 0) S.qn = 0;
      __syncthreads();
      const int64_t c1 = min(ntot, c0 + FMQ);
      for (int64_t i = c0 + threadIdx.x; i < c1; i += ABLOCK) {
        int2 e;
        if (i < n1) {
          e = P[i];
        } else {
          const int64_t k = ls0 + (i - n1);
            e = D.pool[log_addr(D, o, k)];
        }
        if (e.x == W) S.q[atomicAdd(&S.qn, 1)] = e.y;
      }
      __syncthreads();
      nq = S.qn;
    }
    if (c0 == 0) dbg_stamp(D, 14);
    dbg_nq += nq;
    for (int32_t q0 = 0; q0 < nq;) {  // block-uniform rounds, one walked candidate per thread
      int32_t qi = q0 + threadIdx.x;
      FHalf hl, hr;
      bool vl = false, vr = false;
      // a thread whose candidate turns out stale or inside a run (~1/3 of them, known after one or
      // two loads) takes the next candidate past the round's first ABLOCK: a workgroup with a few
      // more candidates than threads walks them in this round instead of a second one (~10 us)
      if (threadIdx.x == 0) S.qsteal = q0 + ABLOCK;
      __syncthreads();
      while (qi < nq && find_walk(D, F, S, S.q[qi], hl, vl, hr, vr)) qi = atomicAdd(&S.qsteal, 1);
      if (c0 == 0 && q0 == 0) dbg_stamp(D, 15);
      // group the new keys of this round: LDS slot, rank within the slot
      bool rl = false, rr = false;
      int32_t sl = -1, sr = -1, kl = 0, kr = 0;
      fkc_group(S, D, vl, hl, sl, rl, kl);
      fkc_group(S, D, vr, hr, sr, rr, kr);
      __syncthreads();
      if (vl && sl >= 0 && S.u.m.kh1[sl] != hl.h1) {  // same probe key, other content
        set_error(D, GEOBPE_EHASH, -13);
        sl = -1;
        vl = false;
      }
      if (vr && sr >= 0 && S.u.m.kh1[sr] != hr.h1) {
        set_error(D, GEOBPE_EHASH, -13);
        sr = -1;
        vr = false;
      }
      {  // exclusive scan of the slot counts -> T offsets
        constexpr int PER = FKC / ABLOCK > 0 ? FKC / ABLOCK : 1;
        int32_t v[PER], sum = 0;
#pragma unroll
        for (int k = 0; k < PER; k++) {
          const int i = threadIdx.x * PER + k;
          v[k] = i < FKC ? S.u.m.kcnt[i] : 0;
          sum += v[k];
        }
        int32_t tot;
        int32_t run = block_excl_scan(sum, &tot, S.red);
#pragma unroll
        for (int k = 0; k < PER; k++) {
          const int i = threadIdx.x * PER + k;
          if (i < FKC) S.u.m.kst[i] = run;
          run += v[k];
        }
        if (threadIdx.x == 0) {
          S.ktot = tot;
          S.fits = (int64_t)S.tb + tot <= D.TC ? 1 : 0;
        }
      }
      __syncthreads();
      if (c0 == 0 && q0 == 0) dbg_stamp(D, 16);
      const bool fits = S.fits != 0;
      const int64_t tbase = (int64_t)r * D.TC + S.tb;
      if (vl) {
        if (sl >= 0 && fits) {
          if (rl) S.u.m.kat[sl] = emit_krec(D, F, S.curK, hl, S.u.m.kcnt[sl], (int32_t)(tbase + S.u.m.kst[sl]));
        } else {
          emit_single(D, F, S.curK, hl);
        }
      }
      if (vr) {
        if (sr >= 0 && fits) {
          if (rr) S.u.m.kat[sr] = emit_krec(D, F, S.curK, hr, S.u.m.kcnt[sr], (int32_t)(tbase + S.u.m.kst[sr]));
        } else {
          emit_single(D, F, S.curK, hr);
        }
      }
      __syncthreads();
      // T entries {occurrence slot, the key's record}: k_place joins them with the record's key
      // id without first loading the record (one dependent round less on the select launch)
      if (vl && sl >= 0 && fits) out_store(&D.T[tbase + S.u.m.kst[sl] + kl], make_int2(hl.target, S.u.m.kat[sl]));
      if (vr && sr >= 0 && fits) out_store(&D.T[tbase + S.u.m.kst[sr] + kr], make_int2(hr.target, S.u.m.kat[sr]));
      if (rl && sl >= 0) {
        S.u.m.kkey[sl] = 0;
        S.u.m.kcnt[sl] = 0;
      }
      if (rr && sr >= 0) {
        S.u.m.kkey[sr] = 0;
        S.u.m.kcnt[sr] = 0;
      }
      if (threadIdx.x == 0 && fits) S.tb += S.ktot;
      __syncthreads();
      q0 = min(S.qsteal, nq);  // (block-uniform: read after the barrier above)
      __syncthreads();  // (before thread 0 resets it for the next round)
    }
  }
  dbg_stamp(D, 12);
  dbg_val(D, 61, dbg_nq + 1);  // (candidates walked, +1)
  dbg_val(D, 62, S.n + 1);     // (occurrences merged, +1)
  // step 1 (the merged pair, -1 on W per occurrence: S.n counts them) and the
  // decrements -> owners
  if (threadIdx.x == 0 && S.n && W >= 0) dec_add(D, F, S.u.m.agg, W, -S.n);
  __syncthreads();
  for (int i = threadIdx.x; i < AggT<12>::N; i += ABLOCK) {
    const int32_t k = S.u.m.agg.key[i], v = S.u.m.agg.val[i];
    if (k < 0 || v == 0) continue;
    const int ow = owner_of_slot(D, (u64)k);
    const int32_t j = atomicAdd(&S.curD[ow], 1);
    if (j < DSH + SD)
      out_store(dec_at(D, (int64_t)ow * D.NBA + r, j), make_int2(k, v));
    else
      global_add(D, k, v, F.to_delta);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < D.NBA; i += ABLOCK) {
    out_store(reinterpret_cast<int2*>(D.cntK) + cnt_at(D, i, r), make_int2(min(S.curK[i], SKR), min(S.curD[i], DSH + SD)));
  }
  if (threadIdx.x == 0) {
    out_store(&D.Lcnt[r], min(S.n, (int32_t)D.LC));
    out_store(&D.Tcnt[r], S.tb);  // (T entries of this region: [r * TC, + Tcnt))
  }
  dbg_stamp(D, 13);
}

// ---------------------------------------------------------------------- k_commit
struct CommitLds;
struct XRes {  // an owner's record reservation (commit_export_reserve -> commit_export)
  int32_t ex;           // this thread's first record within the owner's
  unsigned long long b;  // the owner's base (thread 0: the returning atomic, consumed late)
};
__device__ __attribute__((always_inline)) inline XRes commit_export_reserve(const Dev& D, CommitLds& S);
__device__ __attribute__((always_inline)) inline void commit_export(const Dev& D, CommitLds& S, const XRes& xr);
struct CommitLds {
  union {
    AggT<12> agg;  // decrements of this owner's keys
  } u;
  u64 ckey[CKC];
  u64 ch1[CKC];
  int32_t cn[CKC];     // occurrences of the key (over every finder)
  int32_t cid[CKC];    // key id (-2: resolve failed)
  int32_t cfirst[CKC]; // a record of the key
  u64 ch2[CKC];        // the key's content (for the claim)
  int4 crep[CKC];      // {len, idL, g, idR}
  int32_t preK[NBA_MAX + 1], preD[NBA_MAX + 1];
  int32_t chunk[LOG_CH_MAX + 1];
  int32_t red[ABLOCK / 64];
  int64_t logpos, lognew;
  int32_t nKO, ns, chk, logok, c0, fbn;
};

// segment of a flat index i over NBA prefix sums pre[0..NBA] (pre[w] <= i < pre[w + 1])
__device__ inline int32_t seg_of(const int32_t* pre, int32_t n, int32_t i) {
  int32_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const int32_t mid = (lo + hi) >> 1;
    if (pre[mid] <= i)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// record i of owner j: the fixed slots of finder w, then the overflow list; *at =
// its index in KS, or -(index in KO + 1)
__device__ inline bool commit_rec(const Dev& D, const CommitLds& S, int32_t j, int32_t i, KRec& k, int64_t* at) {
  const int32_t totK = S.preK[D.NBA];
  if (i < totK) {
    const int32_t w = seg_of(S.preK, D.NBA, i);
    *at = krec_at((int64_t)j * D.NBA + w, i - S.preK[w]);
    k = D.KS[*at];
    return true;
  }
  *at = -(int64_t)(i - totK) - 1;
  k = D.KO[i - totK];
  return owner_of_key(D, k.pkey) == j;
}

__device__ inline int32_t ckc_slot(CommitLds& S, u64 k, bool insert, bool* res) {
  int32_t h = (int32_t)((k * 0xD6E8FEB86659FD93ULL) >> (64 - 11)) & (CKC - 1);
  *res = false;
#pragma unroll 1
  for (int probe = 0; probe < 32; probe++, h = (h + 1) & (CKC - 1)) {
    u64 c = S.ckey[h];
    if (c == 0) {
      if (!insert) return -1;
      c = atomicCAS((unsigned long long*)&S.ckey[h], 0ULL, (unsigned long long)k);
      if (c == 0) {
        *res = true;
        return h;
      }
    }
    if (c == k) return h;
  }
  return -1;
}

// key id of a record's content: find or claim in the key table (claim: payload +
// this owner's claim list; find: EHASH check record).  The owner is the only
// workgroup resolving this key in this launch, so the first probe is the CAS itself
// (it returns what the slot holds: empty -> claimed, the key -> found).
__device__ __attribute__((always_inline)) inline int32_t commit_resolve(const Dev& D, CommitLds& S, const KRec& k, bool* claimed_out = nullptr) {
  bool claimed = false;
  const u64 s0 = ht_first_slot(D, k.pkey);
  const u64 old = atomicCAS((unsigned long long*)&D.ht_key[s0], 0ULL, (unsigned long long)k.pkey);
  int32_t d;
  if (old == 0) {
    claimed = true;
    d = (int32_t)s0;
  } else if (old == k.pkey) {
    d = (int32_t)s0;
  } else {
    const u64 s1 = (s0 + 1) & ((u64)D.HC - 1);
    d = ht_resolve(D, k.pkey, s1, ht_probe(D, s1), &claimed);
  }
  if (claimed_out) *claimed_out = claimed;
  if (d < 0) return -1;
  if (claimed) {
    claim_payload(D, d, k.h1, k.h2, k.len, k.idL, k.g, k.idR);
    note_claim(D, &S.ns, d);
  } else {
    emit_check(D, &S.chk, d, k.len, k.h1, k.h2);
  }
  return d;
}

__device__ inline void log_put(const Dev& D, const CommitLds& S, int64_t pos, int32_t d, int32_t slot) {
  const int64_t c = pos / D.CHUNK - S.c0;
  D.pool[(int64_t)S.chunk[c] * D.CHUNK + pos % D.CHUNK] = make_int2(d, slot);
}

// record i past the first PER of each finder's slot (prefix sums preE over finders),
// then the overflow list: its index in KS (KO is KS's tail, from NBA * NBA * SK)
__device__ inline int64_t extra_at(const Dev& D, const int32_t* preE, int32_t nba, int32_t j, int32_t PER, int32_t nE,
                                   int32_t i) {
  if (i < nE) {
    const int32_t ww = seg_of(preE, nba, i);
    return krec_at((int64_t)j * nba + ww, PER + (i - preE[ww]));
  }
  return (int64_t)nba * nba * SK + (i - nE);
}

// commit_resolve with the key's count added in the same round trip: the add to the count of
// the key's first slot goes out beside the CAS (the key is there unless another key took the
// slot first: then the add is undone and the key resolved onward).  An unclaimed slot's count
// is 0, so a claim's count is its occurrence total either way.  The undone add may have hidden
// a theta crossing of the slot's own key from the thread that made it: that key joins the hot
// list unconditionally (a listed key under theta is a stale entry the select skips)
// (the second half: the CAS and the add were issued by the caller, old / c0 their results)
__device__ __attribute__((always_inline)) inline int32_t commit_resolve_finish(const Dev& D, CommitLds& S, HotApp& hot,
                                                                               const KRec& k, int32_t n, int32_t th,
                                                                               u64 s0, u64 old, int32_t c0) {
  bool claimed = false;
  int32_t d;
  if (old == 0 || old == k.pkey) {
    claimed = old == 0;
    d = (int32_t)s0;
    if (th > 0 && c0 < th && c0 + n >= th) hot_push(D, hot, d);
  } else {
    atomicAdd(&D.count[s0], -n);
    if (th > 0) hot_push(D, hot, (int32_t)s0);
    const u64 s1 = (s0 + 1) & ((u64)D.HC - 1);
    d = ht_resolve(D, k.pkey, s1, ht_probe(D, s1), &claimed);
    if (d >= 0) count_add_hot(D, hot, d, n, th);
  }
  if (d < 0) return -1;
  if (claimed) {
    claim_payload(D, d, k.h1, k.h2, k.len, k.idL, k.g, k.idR);
    note_claim(D, &S.ns, d);
  } else {
    emit_check(D, &S.chk, d, k.len, k.h1, k.h2);
  }
  return d;
}

// the key record of table slot s (LDS)
__device__ inline KRec commit_key_at(const CommitLds& S, int32_t s) {
  KRec k;
  k.pkey = S.ckey[s];
  k.h1 = S.ch1[s];
  k.h2 = S.ch2[s];
  const int4 rp = S.crep[s];
  k.len = rp.x;
  k.idL = rp.y;
  k.g = rp.z;
  k.idR = rp.w;
  k.n = S.cn[s];
  k.tstart = 0;
  return k;
}

// a count change k_commit could not stage: a record (pipelined), the global count or the delta
template <bool X>
__device__ inline void commit_add(const Dev& D, int32_t d, int32_t v, bool tod) {
  if (X && tod && D.xrec)
    rec_add(D, d, v);
  else
    global_add(D, d, v, tod);
}

// a record whose key did not fit the dedupe table: resolved and counted on its own
template <bool X>
__device__ __attribute__((always_inline)) inline void commit_fallback(const Dev& D, CommitLds& S, HotApp& hot, const KRec& k, bool tod, int32_t th) {
  const int32_t d = commit_resolve(D, S, k);
  if (d >= 0) {
    atomicAdd(&S.fbn, k.n);
    if (X && tod && D.xrec)
      rec_add(D, d, k.n);
    else if (tod)
      global_add(D, d, k.n, true);
    else
      count_add_hot(D, hot, d, k.n, th);
  }
}

// the key id of a record this owner resolved (-1: none)
__device__ __attribute__((always_inline)) inline int32_t commit_id_of(const Dev& D, CommitLds& S, const KRec& k) {
  bool res;
  const int32_t s = ckc_slot(S, k.pkey, false, &res);
  if (s >= 0) {
    if (S.ch1[s] != k.h1) {  // same probe key, other content
      set_error(D, GEOBPE_EHASH, -13);
      return -1;
    }
    return S.cid[s];
  }
  bool claimed;  // (round 1 resolved it on its own: find it again)
  return ht_resolve(D, k.pkey, ht_first_slot(D, k.pkey), ht_probe(D, ht_first_slot(D, k.pkey)), &claimed);
}

// two records per thread in ONE publish round (r0 and the first extra e0): an owner with a
// single record past a slot's first PER paid a whole second round (block scan, barrier,
// ~3.5 us, profiles/r5_s2/timeline_ab_b.so.txt) -- and such owners end the launch
__device__ __attribute__((always_inline)) inline void commit_publish2(const Dev& D, CommitLds& S, bool m0, const KRec& k0,
                                                                      int64_t at0, bool m1, const KRec& k1, int64_t at1) {
  const int32_t d0 = m0 ? commit_id_of(D, S, k0) : -1, d1 = m1 ? commit_id_of(D, S, k1) : -1;
  const int32_t n0 = m0 && d0 >= 0 ? k0.n : 0, n1 = m1 && d1 >= 0 ? k1.n : 0;
  int32_t tot;
  const int32_t ex = block_excl_scan(n0 + n1, &tot, S.red);
  if (m0) *rec_id(D, at0) = make_int2(d0 >= 0 ? d0 : -1, S.logok && d0 >= 0 ? (int32_t)(S.logpos + ex) : -1);
  if (m1) *rec_id(D, at1) = make_int2(d1 >= 0 ? d1 : -1, S.logok && d1 >= 0 ? (int32_t)(S.logpos + ex + n0) : -1);
  __syncthreads();
  if (threadIdx.x == 0) S.logpos += tot;
}

// a record's key id and posting-log position (block-uniform: every thread calls it)
__device__ __attribute__((always_inline)) inline void commit_publish(const Dev& D, CommitLds& S, bool mine, const KRec& k, int64_t at) {
  const int32_t d = mine ? commit_id_of(D, S, k) : -1;
  const int32_t n = mine && d >= 0 ? k.n : 0;
  int32_t tot;
  const int32_t ex = block_excl_scan(n, &tot, S.red);
  if (mine) {
    const int2 v = make_int2(d >= 0 ? d : -1, S.logok && d >= 0 ? (int32_t)(S.logpos + ex) : -1);
    *rec_id(D, at) = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) S.logpos += tot;
}

// pipelined exchange: this owner's delta records -- every resolved key with its
// occurrence total, every decremented key with its (negative) total, and its share of
// k_find's side list -- straight into the rank's slot, one reservation per workgroup on
// the slot header's count (final when k_commit ends: no header pass).  The producer applies
// its own rank's deltas at once (x_put_rec); the imports add the other ranks' records.
// (two halves: the count and the reservation right after the resolves -- the returning atomic
// then completes under the publish rounds instead of after them; the stores at the end)
__device__ __attribute__((always_inline)) inline XRes commit_export_reserve(const Dev& D, CommitLds& S) {
  const int t = threadIdx.x;
  const int64_t nx = min(D.st->nxovf, D.KCAP);  // (k_find's; k_commit adds none)
  const int64_t x0 = nx * blockIdx.x / gridDim.x, x1 = nx * (blockIdx.x + 1) / gridDim.x;
  int32_t c = 0;
  for (int32_t s = t; s < CKC; s += ABLOCK) c += S.ckey[s] != 0 && S.cid[s] >= 0;
  for (int i = t; i < AggT<12>::N; i += ABLOCK) c += S.u.agg.key[i] >= 0 && S.u.agg.val[i] != 0;
  for (int64_t i = x0 + t; i < x1; i += ABLOCK) c++;
  int32_t tot;
  XRes r;
  r.ex = block_excl_scan(c, &tot, S.red);
  r.b = t == 0 && tot ? atomicAdd((unsigned long long*)(D.xcnt ? D.xcnt : &D.st->ntouched), (unsigned long long)tot) : 0ULL;
  return r;
}
__device__ __attribute__((always_inline)) inline void commit_export(const Dev& D, CommitLds& S, const XRes& xr) {  // (inlined: a call takes D's address, and the whole Dev goes to scratch)
  __shared__ unsigned long long s_xb;
  const int t = threadIdx.x;
  const int64_t nx = min(D.st->nxovf, D.KCAP);
  const int64_t x0 = nx * blockIdx.x / gridDim.x, x1 = nx * (blockIdx.x + 1) / gridDim.x;
  if (t == 0) s_xb = xr.b;
  __syncthreads();
  const int32_t ex = xr.ex;
  int64_t j = (int64_t)s_xb + ex;
  for (int32_t s = t; s < CKC; s += ABLOCK) {
    if (S.ckey[s] == 0 || S.cid[s] < 0) continue;
    const int4 rp = S.crep[s];
    DeltaRec r;
    r.h1 = S.ch1[s];
    r.h2 = S.ch2[s];
    r.len = rp.x;
    r.idL = rp.y;
    r.g = rp.z;
    r.idR = rp.w;
    r.delta = S.cn[s];
    r.pad = S.cid[s] + 1;  // (this rank's key id: x_put_rec applies the delta by it, no probe)
    x_put_rec(D, j, r, -30);
    j++;
  }
  auto put_id = [&](int32_t k, int32_t v) {
    DeltaRec r;
    r.h1 = D.kh1[k];
    r.h2 = D.kh2[k];
    r.len = D.klen[k];
    r.idL = D.krep[3 * (int64_t)k];
    r.g = D.krep[3 * (int64_t)k + 1];
    r.idR = D.krep[3 * (int64_t)k + 2];
    r.delta = v;
    r.pad = k + 1;
    x_put_rec(D, j, r, -30);
    j++;
  };
  for (int i = t; i < AggT<12>::N; i += ABLOCK) {
    const int32_t k = S.u.agg.key[i], v = S.u.agg.val[i];
    if (k >= 0 && v != 0) put_id(k, v);
  }
  for (int64_t i = x0 + t; i < x1; i += ABLOCK) {
    const int2 e = D.xovf[i];
    put_id(e.x, e.y);
  }
}

template <bool X>
__device__ __attribute__((always_inline)) inline void commit_main(const Dev& D, int to_delta, int par) {
  __shared__ CommitLds S;
  __shared__ HotApp hot;
  __shared__ int64_t s_kl[2];
  __shared__ int32_t s_preE[NBA_MAX + 1], s_preF[NBA_MAX + 1];
  __shared__ TouchBuf tb;
  State* st = D.st;
  if (par < 0) {  // pipelined exchange (k_select set dgen)
    if (st->stall) return;
    par = st->dgen & 1;
  }
  const int32_t j = blockIdx.x;
  // ---- one round of loads for everything that depends only on j: the record
  // counts of every finder and, speculatively, the first PER records of each
  // finder's slot (a finder sends an owner ~1-2 records in the heavy merges), the
  // same for the decrement records, the log cursor, the state
  const int32_t nba = D.NBA;
  const int32_t PER = ABLOCK / nba;  // >= 4 (NBA <= 256)
  const int32_t t = threadIdx.x;
  const int32_t w = t % nba, k0 = t / nba;
  const bool lane_ok = k0 < PER;
  const int64_t seg = (int64_t)j * nba + w;
  const int2 cKD = cnt_pair(D, j, w);
  const int32_t cK = cKD.x, cD = cKD.y;
  const Sel sel = D.sel[par];
  const int32_t th = st->theta;
  const int32_t pn = D.pnch[j], pf = D.pfill[j];
  const int32_t plog_ovf0 = st->plog_ovf;  // (read with the first round: the log reservation needs it)
  const int64_t nko_raw = st->nko2[par];
  const int64_t novf_raw = j == 0 ? st->L_ovf2[par] : 0;
  const int64_t kl0 = D.kchunk[2 * j], kl1 = D.kchunk[2 * j + 1];  // (this owner's klist chunk)
  int32_t lc = 0;
  if (j == 0 && t < nba) lc = D.Lcnt[t];
  if (j == 0 && t == 0) {
    st->L_ovf2[par ^ 1] = 0;  // the next find's overflow counters (idle since the last pair)
    st->nko2[par ^ 1] = 0;
    st->place_par = sel.decision == SEL_MERGE ? par : -1;  // k_place's merge (with the next select)
    st->place_nid = sel.nid;
    st->place_novf = min(novf_raw, D.Lovf_cap);
    st->place_nko = min(nko_raw, D.KO_cap);
    if (sel.decision == SEL_DONE) {
      st->done = 1;
      st->maxc = 0;
    } else if (sel.decision == SEL_SKIP) {
      st->nskip += 1;
    }
  }
  if (sel.decision == SEL_DONE || sel.decision == SEL_IDLE) return;
  if (sel.decision == SEL_SKIP) {
    if (sel.skip & SKIP_MEASURE) measure_max(D);
    if (sel.skip & SKIP_HOT) rebuild_hot_list(D, sel.theta_new, sel.build);
    return;
  }
  dbg_stamp(D, 0);
  const bool tod = to_delta != 0;
  const int32_t nid = sel.nid;
  if (j == 0) {  // _tokens[n] = json.loads(key): content(L) ++ [g] ++ content(R)
    const int32_t L = sel.widL, g = sel.wg, Rr = sel.widR;
    const int64_t vL = D.voff[L], vR = D.voff[Rr];
    const int64_t nL = D.voff[L + 1] - vL, nR = D.voff[Rr + 1] - vR;
    const int64_t pos = D.voff[nid], ln = nL + 1 + nR;
    if (pos + ln > D.VSC) {
      if (t == 0) set_error(D, GEOBPE_ECAPACITY, -9);
    } else {
      for (int64_t i = t; i < ln; i += blockDim.x)
        D.vsym[pos + i] = i < nL ? D.vsym[vL + i] : (i == nL ? g : D.vsym[vR + i - nL - 1]);
      if (t == 0) D.voff[nid + 1] = pos + ln;
    }
  }
  dbg_stamp(D, 50);
  for (int i = t; i < CKC; i += ABLOCK) {
    S.ckey[i] = 0;
    S.cn[i] = 0;
  }
  for (int i = t; i < AggT<12>::N; i += ABLOCK) {
    S.u.agg.key[i] = -1;
    S.u.agg.val[i] = 0;
  }
  hot_init(hot);
  if (t == 0) tb.n = 0;
  dbg_stamp(D, 51);
  {  // records past the first PER of a finder's slot: prefix sums
    const int32_t eK = t < nba ? max(0, min(cK, SKR) - PER) : 0;
    const int32_t eD = t < nba ? max(0, min(cD, DSH + SD) - PER) : 0;
    int32_t totE, totF;
    const int32_t xE = block_excl_scan(eK, &totE, S.red);
    const int32_t xF = block_excl_scan(eD, &totF, S.red);
    if (t < nba) {
      s_preE[t] = xE;
      s_preF[t] = xF;
    }
    if (t == 0) {
      s_preE[nba] = totE;
      s_preF[nba] = totF;
      S.nKO = (int32_t)min(nko_raw, D.KO_cap);
      S.ns = 0;
      S.chk = 0;
      S.fbn = 0;
      s_kl[0] = kl0;
      s_kl[1] = kl1;
    }
  }
  __syncthreads();
  dbg_stamp(D, 1);
  // the first PER records of each finder's slot, only where they exist (issuing them before the
  // prefix scans above measured ~1 % slower on the window, profiles/r5_s5/)
  KRec r0;
  int2 d0 = make_int2(0, 0);
  // (unconditional loads from clamped slots, all of this round's loads issued before any wait: a
  // load inside `if` made the compiler wait for it at the join, r0 / d0 / e0 / x0 one after another)
  {
    const bool hk = lane_ok && k0 < min(cK, SKR), hd = lane_ok && k0 < min(cD, DSH + SD);
    r0 = ld_rec(&D.KS[krec_at(seg, hk ? k0 : 0)]);
    const int2 d0r = ld_now(dec_at(D, seg, hd ? k0 : 0));
    d0 = hd ? d0r : make_int2(0, 0);
  }
  // ---- round 1: key records -> LDS dedupe (occurrence totals per key); decrements -> LDS
#define COMMIT_INSERT(k)                                          \
  do {                                                            \
    bool res_;                                                    \
    const int32_t s_ = ckc_slot(S, (k).pkey, true, &res_);        \
    if (s_ >= 0) {                                                \
      if (res_) {                                                 \
        S.ch1[s_] = (k).h1;                                       \
        S.ch2[s_] = (k).h2;                                       \
        S.crep[s_] = make_int4((k).len, (k).idL, (k).g, (k).idR); \
      }                                                           \
      atomicAdd(&S.cn[s_], (k).n);                                \
    } else {                                                      \
      commit_fallback<X>(D, S, hot, (k), tod, th);                   \
    }                                                             \
  } while (0)
  const bool mine0 = lane_ok && k0 < min(cK, SKR);
  const int32_t nE = s_preE[nba], nF = s_preF[nba], nKO = S.nKO;
  // this thread's first record past a slot's first PER (extras, then the overflow list) and
  // its first extra decrement record go out in the same round as r0 / d0: the owners with
  // extras -- the ones holding the most hot keys, which end the launch -- paid one more
  // dependent round trip for them (~3 us, profiles/r4_final/merge_timeline_heavy.txt).  The
  // first extra stays in registers for the publish round as well.
  KRec e0;
  int64_t at0 = 0;
  const bool he = t < nE + nKO;
  int2 x0 = make_int2(-1, 0);
  {
    if (he) at0 = extra_at(D, s_preE, nba, j, PER, nE, t);
    const int2* xa = D.DS;
    if (t < nF) {
      const int32_t ww = seg_of(s_preF, nba, t);
      xa = dec_at(D, (int64_t)j * nba + ww, PER + (t - s_preF[ww]));
    }
    e0 = ld_rec(&D.KS[at0]);
    const int2 x0r = ld_now(xa);
    x0 = t < nF ? x0r : make_int2(-1, 0);
  }
  if (mine0) COMMIT_INSERT(r0);
  if (lane_ok && k0 < min(cD, DSH + SD) && !agg_stage(S.u.agg, d0.x, d0.y)) commit_add<X>(D, d0.x, d0.y, tod);
  dbg_stamp(D, 56);
  if (he && (t < nE || owner_of_key(D, e0.pkey) == j)) COMMIT_INSERT(e0);
  for (int32_t i = t + ABLOCK; i < nE + nKO; i += ABLOCK) {  // (rare: more than ABLOCK extras)
    const KRec k = D.KS[extra_at(D, s_preE, nba, j, PER, nE, i)];
    if (i < nE || owner_of_key(D, k.pkey) == j) COMMIT_INSERT(k);
  }
  dbg_stamp(D, 57);
  dbg_val(D, 59, nF);
  if (t < nF && !agg_stage(S.u.agg, x0.x, x0.y)) commit_add<X>(D, x0.x, x0.y, tod);
  for (int32_t i = t + ABLOCK; i < nF; i += ABLOCK) {
    const int32_t ww = seg_of(s_preF, nba, i);
    const int2 x = *dec_at(D, (int64_t)j * nba + ww, PER + (i - s_preF[ww]));
    if (!agg_stage(S.u.agg, x.x, x.y)) commit_add<X>(D, x.x, x.y, tod);
  }
  dbg_stamp(D, 58);
  __syncthreads();
  dbg_stamp(D, 2);
  if (D.dbg) {  // (debug timeline: this owner's work, block-uniform)
    const int32_t nr = __syncthreads_count(mine0), nd = __syncthreads_count(lane_ok && k0 < min(cD, DSH + SD));
    dbg_val(D, 7, nr + nE + nKO);
    dbg_val(D, 8, nd + nF);
  }
  // ---- posting-log space for this merge's new pairs of this owner (one reservation), sized from
  // round 1's occurrence totals (a key that then fails to resolve only leaves its space unused):
  // the reservation's returning atomic on the pool cursor is in flight under the resolves, not
  // after them (~2-4 us on the owners that open a chunk)
  int64_t lbase = 0;
  int32_t lneed = 0, lc1 = 0;
  {
    int32_t mine_n = 0;
    for (int32_t s = t; s < CKC; s += ABLOCK) mine_n += S.ckey[s] != 0 ? S.cn[s] : 0;
    int32_t tot;
    block_excl_scan(mine_n, &tot, S.red);
    if (t == 0) {
      const int64_t add = (int64_t)tot + S.fbn;  // (+ records whose key did not fit the dedupe table)
      const int64_t p0 = pn > 0 ? (int64_t)(pn - 1) * D.CHUNK + pf : 0;
      S.logpos = p0;
      S.logok = 0;
      lc1 = (int32_t)((p0 + add + D.CHUNK - 1) / D.CHUNK);  // chunks [0, lc1) hold the log
      if (!plog_ovf0 && lc1 - (int32_t)(p0 / D.CHUNK) <= LOG_CH_MAX && lc1 <= D.MAXCH) {
        lneed = max(0, lc1 - pn);
        lbase = lneed ? (int64_t)atomicAdd((unsigned long long*)&st->pool_used, (unsigned long long)lneed) : 0;
      } else {
        lneed = -1;
      }
    }
  }
  // ---- every distinct key once: find or claim, its count (+ hot-list crossing)
  int32_t nkeys = 0;
  if (!tod) {
    // this thread's two table slots: both keys' CAS and count add out before any result is used
    static_assert(CKC == 2 * ABLOCK, "two commit table slots per thread");
    const u64 ka = S.ckey[t], kb = S.ckey[t + ABLOCK];
    const int32_t na = S.cn[t], nb = S.cn[t + ABLOCK];
    const u64 sa = ht_first_slot(D, ka), sb = ht_first_slot(D, kb);
    u64 oa = 0, ob = 0;
    int32_t ca = 0, cb = 0;
    if (ka) {
      oa = atomicCAS((unsigned long long*)&D.ht_key[sa], 0ULL, (unsigned long long)ka);
      ca = atomicAdd(&D.count[sa], na);
    }
    if (kb) {
      ob = atomicCAS((unsigned long long*)&D.ht_key[sb], 0ULL, (unsigned long long)kb);
      cb = atomicAdd(&D.count[sb], nb);
    }
    if (ka) {
      const int32_t d = commit_resolve_finish(D, S, hot, commit_key_at(S, t), na, th, sa, oa, ca);
      S.cid[t] = d >= 0 ? d : -2;
      if (d >= 0) nkeys++;
    }
    if (kb) {
      const int32_t d = commit_resolve_finish(D, S, hot, commit_key_at(S, t + ABLOCK), nb, th, sb, ob, cb);
      S.cid[t + ABLOCK] = d >= 0 ? d : -2;
      if (d >= 0) nkeys++;
    }
  }
  for (int32_t s = t; s < CKC && tod; s += ABLOCK) {
    const u64 key = S.ckey[s];
    if (key == 0) continue;
    KRec k;
    k.pkey = key;
    k.h1 = S.ch1[s];
    k.h2 = S.ch2[s];
    const int4 rp = S.crep[s];
    k.len = rp.x;
    k.idL = rp.y;
    k.g = rp.z;
    k.idR = rp.w;
    const int32_t n = S.cn[s];
    bool claimed;
    const int32_t d = commit_resolve(D, S, k, &claimed);
    if (d >= 0 && !tod) count_add_hot(D, hot, d, n, th);
    S.cid[s] = d >= 0 ? d : -2;
    if (d >= 0) {
      if (tod && !(X && D.xrec)) touch_add(D, tb, d, n);  // (direct records: written below)
      nkeys++;
    }
  }
  XRes xres{0, 0ULL};
  if constexpr (X) {
    if (tod && D.xrec) xres = commit_export_reserve(D, S);  // (block-uniform: every key resolved, the decrements staged)
  }
  // ---- decrements of this owner's keys: one atomic per key, in flight under the log
  // reservation and the publish round (a decrement cannot hide a theta crossing: a positive
  // add that follows sees less; before the resolves they queued ahead of them)
  if (!tod)
    for (int i = t; i < AggT<12>::N; i += ABLOCK) {
      const int32_t k = S.u.agg.key[i], v = S.u.agg.val[i];
      if (k >= 0 && v != 0) atomicAdd(&D.count[k], v);
    }
  if (D.dbg) {
    int32_t tk;
    block_excl_scan(nkeys, &tk, S.red);
    dbg_val(D, 9, tk);
  }
  if (D.stats) {  // (profiling: the work of this launch, for the bench's algorithmic bytes)
    int32_t tk, tr, td;
    block_excl_scan(nkeys, &tk, S.red);
    block_excl_scan(mine0 ? 1 : 0, &tr, S.red);
    block_excl_scan(lane_ok && k0 < min(cD, DSH + SD) ? 1 : 0, &td, S.red);
    if (t == 0) {
      atomicAdd((unsigned long long*)&st->stat_keys, (unsigned long long)tk);
      atomicAdd((unsigned long long*)&st->stat_krec, (unsigned long long)(tr + nE + nKO));
      atomicAdd((unsigned long long*)&st->stat_drec, (unsigned long long)(td + nF));
    }
  }
  // the reservation made before the resolves: the new chunks into the owner's chunk table
  if (t == 0) {
    if (lneed >= 0 && lbase + lneed <= D.POOL_CH) {
      for (int32_t c = pn; c < lc1; c++) D.pch[(int64_t)j * D.MAXCH + c] = (int32_t)(lbase + (c - pn));
      S.logok = 1;
    }
    if (!S.logok) st->plog_ovf = 1;  // the next merge rebuilds the posting index first
  }
  __syncthreads();
  dbg_stamp(D, 3);
  // ---- round 2: every record's key id and posting-log position (k_place writes pk
  // and the log entries of its occurrence slots); the first PER records per finder
  // are still in registers
  commit_publish2(D, S, mine0, r0, krec_at(seg, k0),he && (t < nE || owner_of_key(D, e0.pkey) == j), e0, at0);
  dbg_stamp(D, 53);
  dbg_val(D, 54, nE);
  dbg_val(D, 55, nKO);
  for (int32_t i0 = ABLOCK; i0 < nE + nKO; i0 += ABLOCK) {  // block-uniform (rare: more than ABLOCK extras)
    const int32_t i = i0 + t;
    const bool in = i < nE + nKO;
    KRec k;
    int64_t at = 0;
    if (in) {
      at = extra_at(D, s_preE, nba, j, PER, nE, i);
      k = D.KS[at];
    }
    const bool mine = in && (i < nE || owner_of_key(D, k.pkey) == j);
    commit_publish(D, S, mine, k, at);
  }
  dbg_stamp(D, 4);
  // ---- decrements of this owner's keys (multi-rank: into the touched list / the records)
  if (tod && !(X && D.xrec))
    for (int i = t; i < AggT<12>::N; i += ABLOCK) {
      const int32_t k = S.u.agg.key[i], v = S.u.agg.val[i];
      if (k >= 0 && v != 0) touch_add(D, tb, k, v);
    }
  if (tod && !(X && D.xrec)) touch_flush(D, tb);  // (block-uniform)
  if constexpr (X) {
    if (tod && D.xrec) commit_export(D, S, xres);  // (block-uniform)
  }
  hot_flush(D, hot);  // (syncs the workgroup first)
  if (t == 0) {
    D.chkcnt[j] = min(S.chk, (int32_t)D.RC);
    if (S.logok) {
      const int64_t end = S.logpos;
      const int32_t nc = (int32_t)((end + D.CHUNK - 1) / D.CHUNK);
      if (end > 0) {
        D.pnch[j] = nc;
        D.pfill[j] = (int32_t)(end - (int64_t)(nc - 1) * D.CHUNK);
      }
    }
  }
  // this owner's claims join klist from its chunk (a reservation only when the chunk
  // runs out; the chunk state was read at kernel start)
  __syncthreads();
  {
    const int32_t n = min(S.ns, (int32_t)D.RC);
    if (t == 0 && n) {
      if (s_kl[1] - s_kl[0] < n) {
        const int64_t sz = max((int64_t)KL_CHUNK, (int64_t)n);
        s_kl[0] = (int64_t)atomicAdd((unsigned long long*)&st->U, (unsigned long long)sz);
        s_kl[1] = s_kl[0] + sz;
      }
      D.kchunk[2 * j] = s_kl[0] + n;
      D.kchunk[2 * j + 1] = s_kl[1];
    }
    __syncthreads();
    const int32_t* reg = D.ns + (int64_t)j * D.RC;
    for (int32_t i = t; i < n; i += blockDim.x) klist_put(D, s_kl[0] + i, reg[i]);
  }
  dbg_stamp(D, 5);
  if (j == 0) {  // merges made this iteration -> merge log, state (k_select reads iter / K)
    int32_t tot;
    block_excl_scan(lc, &tot, S.red);
    if (t == 0) {
      const int64_t novf = min(st->L_ovf2[par], D.Lovf_cap);
      D.log[sel.iter].nmerged = (int64_t)tot + novf;
      st->iter = sel.iter + 1;
      st->K = sel.nid + 1;
      st->maxc = sel.maxc;
      st->ncand = sel.ncand;
    }
  }
  dbg_stamp(D, 6);
}

// X: the pipelined exchange's instantiation (the record export, the peer exchange's arrival); the
// one-rank loop's carries none of that code (round 6's first form: +1.6 us a launch, its SGPR
// spills 102 -> 276 from the peer pointers held for the export)
template <bool X>
__global__ __launch_bounds__(ABLOCK) void k_commit(Dev D, int to_delta, int par) {
  commit_main<X>(D, to_delta, par);
  if constexpr (X) x_arrive(D);  // (the peer exchange: this launch's records are out, exchange.h)
}

// ---------------------------------------------------------------------- k_place
// Region j's half of the merge after its keys are resolved: the token rewrites of
// find region j (step 2, bond_to_token / token_pos: tok[a] = {X, |X|}, b stops
// being a token start, c's previous token is a) and, for every key record finder j
// sent (and its share of the overflow list), pk of the occurrence slots and their
// posting-log entries -- balanced by region, whatever the key skew.
struct PlaceLds {
  int32_t pre[NBA_MAX + 1];
  int32_t red[ABLOCK / 64];
};

// the owner whose posting log a record's occurrences join: the owner slot of a KS index, the
// key's owner for an overflow record (KO, KS's tail)
__device__ inline int32_t place_owner(const Dev& D, int32_t at) {
  const int64_t base = (int64_t)D.NBA * D.NBA * SK;
  return at < base ? (int32_t)(at / ((int64_t)D.NBA * SK)) : owner_of_key(D, D.KS[at].pkey);
}

// record i of finder region j's records (the owners' slots, then its share k_lo.. of the
// overflow list): its KS index
__device__ inline int32_t place_rec_at(const Dev& D, const PlaceLds& S, int32_t j, int32_t i, int32_t nk, int64_t k_lo) {
  if (i < nk) {
    const int32_t ow = seg_of(S.pre, D.NBA, i);
    return (int32_t)krec_at((int64_t)ow * D.NBA + j, i - S.pre[ow]);
  }
  return (int32_t)((int64_t)D.NBA * D.NBA * SK + k_lo + (i - nk));
}


// k_place's token rewrites, pk and posting-log entries (read by the next k_find on every XCD):
// PLACE_WT=1 stores them write-through (A/B)
template <typename V>
__device__ inline void pl_store(V* p, const V& v) {
  *p = v;
}

// the token rewrites of one merged occurrence (a, b) with right neighbour c: a becomes the new
// token, b's record is cleared, c's previous slot is a (or a ends its chain)
__device__ inline void place_tokens(const Dev& D, const LEntry& e, int32_t nid) {
  pl_store(reinterpret_cast<int2*>(D.tok + e.a), make_int2(nid, e.ya));
  pl_store(D.tok + e.b, make_int4(-1, 0, -1, -1));  // (no other occurrence writes b's record)
  if (e.c >= 0)
    pl_store(tok_f(D, e.c, 2), e.a);
  else
    pl_store(tok_f(D, e.a, 3), (int32_t)-1);
}

// a single record (one occurrence, its slot in tstart as -(slot + 1)) of finder region j: pk
// of the slot and its posting-log entry.  Grouped records are written through their T entries.
__device__ inline void place_single(const Dev& D, int32_t at, int2 nt, int2 v) {
  if (nt.y >= 0 || v.x < 0) return;
  const int32_t t = -(nt.y + 1);
  pl_store(tok_f(D, t, 3), v.x);
  if (v.y >= 0) pl_store(&D.pool[log_addr(D, place_owner(D, at), v.y)], make_int2(v.x, t));
}

// T entry {slot, record} at T index q: pk of the slot and its posting-log entry (its position
// in the record's range: the record's log position + q - tstart)
__device__ inline void place_tentry(const Dev& D, int64_t q, int2 e, int2 v, int32_t tstart) {
  if (e.y < 0 || v.x < 0) return;
  pl_store(tok_f(D, e.x, 3), v.x);
  if (v.y >= 0) pl_store(&D.pool[log_addr(D, place_owner(D, e.y), (int64_t)v.y + (q - tstart))], make_int2(v.x, e.x));
}

// place the merge committed with launch parity st->place_par (k_commit sets it; -1:
// nothing to place).  Idempotent until the next k_find: a re-run writes the same
// values (the pipelined exchange may run it again behind a stall).
//
// Two dependent rounds of loads.  Round 1: the merge's header (k_commit's copy in the state),
// this region's merge entries, the record counts finder j sent each owner, and its T entries
// {occurrence slot, key record} (up to 2 per thread).  Round 2: every record's (n, tstart) and
// (key id, log position), and for every T entry its record's (key id, log position) and tstart
// -- the T entries carry their record, so they need no record first (round 4's place loaded the
// records, then the T ranges: three rounds on the select launch's critical path).
__device__ void place_body(const Dev& D, int32_t j, PlaceLds& S) {
  State* st = D.st;
  const int32_t t = threadIdx.x;
  const int32_t par = st->place_par;
  const int32_t nid = st->place_nid;
  const int64_t novf = st->place_novf, nko = st->place_nko;
  const int32_t nA = D.Lcnt[j];
  const LEntry eA = D.L[(int64_t)j * D.LC + min((int64_t)t, D.LC - 1)];
  const int32_t cK = t < D.NBA ? cnt_pair(D, t, j).x : 0;
  const int32_t nT = min((int64_t)D.Tcnt[j], D.TC);
  const int2* Tj = D.T + (int64_t)j * D.TC;
  const int2 te0 = Tj[min(t, (int32_t)D.TC - 1)], te1 = Tj[min(t + ABLOCK, (int32_t)D.TC - 1)];
  if (par < 0) return;  // (k_commit sets par only for a merge)
  dbg_stamp(D, 30);
  // ---- round 2, part 1: every T entry's record (key id, log position, tstart) -- they need only
  // round 1's T entries, so they go out before the scan below (issued after it, behind the
  // records' loads, the compiler waited for each group in turn: three round trips, ~4.5 us)
  // (unconditional loads from a clamped index: a load inside `if` into a register the other path
  // sets made the compiler wait for it at the join, one group after the other)
  const bool h0 = t < nT && te0.y >= 0, h1 = t + ABLOCK < nT && te1.y >= 0;
  const int32_t a0 = h0 ? te0.y : 0, a1 = h1 ? te1.y : 0;
  const int4 q0 = rec_tail(D, a0), q1 = rec_tail(D, a1);
  const int2 v0 = h0 ? make_int2(q0.x, q0.y) : make_int2(-1, -1), v1 = h1 ? make_int2(q1.x, q1.y) : make_int2(-1, -1);
  const int32_t ts0 = h0 ? q0.w : 0, ts1 = h1 ? q1.w : 0;
  const int64_t oper = (novf + D.NBA - 1) / D.NBA;
  const int64_t o_lo = (int64_t)j * oper, o_n = max((int64_t)0, min(novf, o_lo + oper) - o_lo);
  const int64_t kper = (nko + D.NBA - 1) / D.NBA;
  const int64_t k_lo = (int64_t)j * kper, k_n = max((int64_t)0, min(nko, k_lo + kper) - k_lo);
  {
    int32_t tot;
    const int32_t e = block_excl_scan(cK, &tot, S.red);
    if (threadIdx.x < D.NBA) S.pre[threadIdx.x] = e;
    if (threadIdx.x == 0) S.pre[D.NBA] = tot;
  }
  __syncthreads();  // S.pre
  dbg_stamp(D, 38);
  const int32_t nk = S.pre[D.NBA];
  const int32_t nrec = nk + (int32_t)k_n;
  // ---- round 2, part 2: the records of this finder's slots (their ranges need the scan)
  const bool hr = t < nrec;
  const int32_t ra = hr ? place_rec_at(D, S, j, t, nk, k_lo) : 0;
  const int4 rq = rec_tail(D, ra);
  const int2 rnt = hr ? make_int2(rq.z, rq.w) : make_int2(0, 0), rv = hr ? make_int2(rq.x, rq.y) : make_int2(-1, -1);
  dbg_stamp(D, 37);
  // ---- the token rewrites of find region j (round 1's data).  The thread's first entry comes from
  // registers with no load on its path (a conditional load there made the compiler wait for every
  // outstanding load, round 2's included, before the first store); the rest -- more entries than
  // threads, the overflow list -- are rare
  if (t < nA) place_tokens(D, eA, nid);
  for (int64_t i = t + ABLOCK; i < nA; i += ABLOCK) place_tokens(D, D.L[(int64_t)j * D.LC + i], nid);
  for (int64_t i = t; i < o_n; i += ABLOCK) place_tokens(D, D.Lovf[o_lo + i], nid);
  dbg_stamp(D, 31);
  // ---- pk of every new pair and its posting-log entry
  const int64_t qbase = (int64_t)j * D.TC;
  if (t < nrec) place_single(D, ra, rnt, rv);
  if (h0) place_tentry(D, qbase + t, te0, v0, ts0);
  if (h1) place_tentry(D, qbase + t + ABLOCK, te1, v1, ts1);
  for (int32_t i = t + ABLOCK; i < nrec; i += ABLOCK) {  // (rare: more records than threads)
    const int32_t at = place_rec_at(D, S, j, i, nk, k_lo);
    const int4 q = rec_tail(D, at);
    place_single(D, at, make_int2(q.z, q.w), make_int2(q.x, q.y));
  }
  for (int32_t q = t + 2 * ABLOCK; q < nT; q += ABLOCK) {  // (rare: more than 2 per thread)
    const int2 e = Tj[q];
    if (e.y >= 0) {
      const int4 r = rec_tail(D, e.y);
      place_tentry(D, qbase + q, e, make_int2(r.x, r.y), r.w);
    }
  }
  dbg_stamp(D, 32);
}

__global__ __launch_bounds__(ABLOCK) void k_place(Dev D) {
  __shared__ PlaceLds S;
  // (the standalone launch flushes a run's last place, usually already done by an idle
  // iteration's select launch: nothing to wait for then -- the place's own first round of
  // loads took ~13 us to drain before its workgroups could see par < 0)
  if (D.st->place_par < 0) return;
  place_body(D, blockIdx.x, S);
}
