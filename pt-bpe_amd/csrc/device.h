// device.h -- device-side data layout and helpers of the GeoBPE engine (gfx950).
// Included once, by geobpe.hip.  See DESIGN.md §3 for the layout rationale.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/geobpe.h"

typedef unsigned long long u64;

namespace gb {

constexpr u64 M61 = (1ULL << 61) - 1;
constexpr u64 HP1 = 0x0A3B5C7D9E1F2437ULL % M61;  // content-hash bases (< M61)
constexpr u64 HP2 = 0x13579BDF2468ACE1ULL % M61;
constexpr u64 KMIX = 0x9E3779B97F4A7C15ULL;
constexpr double TWO_PI = 6.283185307179586;  // 2*np.pi
constexpr int BLOCK = 256;
constexpr int ABLOCK = 1024;  // region kernels (bin pairs, finalize, apply, import): 16 waves per CU
constexpr int CL_MIN_SHRINK = 4096;  // hot-list length above which a 4x drop of theta re-scans
constexpr int PIPE_MAX_WORLD = 64;  // ranks of a pipelined exchange
constexpr int XPEER_MAX = 8;        // peer exchange: ranks (one node)
constexpr int XHDR = 64;            // peer exchange: slot header bytes {int64 count, int32 seq}
constexpr int NBKT_LOG2 = 14;        // key buckets of the posting index (per region)
constexpr int NBKT = 1 << NBKT_LOG2;
constexpr int SKIP_HOT = 1, SKIP_MEASURE = 4;  // what a rebuild iteration does
constexpr int DBG_SLOTS = 64;
constexpr int PW_LDS = 2048;  // hash powers staged in LDS by k_apply (chains up to ~1000 residues)
constexpr int KL_CHUNK = 4096;  // klist entries a commit workgroup reserves at a time
// merge find -> commit hand-off (merge.h): per (owner, find workgroup) fixed record
// slots, overflow to one global list
constexpr int NBA_MAX = 256;
constexpr int SK = 48;      // key-record slots per (owner, find workgroup); slot 0 holds decrements (below)
constexpr int SD = 48;      // decrement records per (owner, find workgroup) past the DSH in slot 0
constexpr int FKC = 2048;   // find: new-key dedupe slots (LDS) per round
constexpr int CKC = 2048;   // commit: key dedupe slots (LDS) per owner
constexpr int FMQ = 4096;    // find: candidate queue (LDS) per chunk of posting entries
constexpr int LOG_CH_MAX = 64;  // posting-log chunks one owner may add in one merge

// ------------------------------------------------------------------ records
// Kernel-to-kernel state.  No field is written by a kernel that other
// workgroups of the same kernel read: k_mark reads State and writes only Sel
// (its workgroup 0); k_apply reads Sel and its workgroup 0 writes State.
struct State {
  // persistent
  int64_t U;          // klist entries reserved (keys + unused chunk tails)
  int64_t nkeys;      // keys
  int64_t err_code;   // first error (GEOBPE_E*)
  int64_t err_pos;
  int64_t epoch;      // delta-touch epoch (multi-rank)
  int32_t K;          // len(_tokens) on the device
  int32_t iter;       // merges made so far
  int32_t done;       // 1 once no pair is left
  int32_t maxc, ncand;  // the last merge's count and tied keys (stats)
  int32_t stall;      // pipelined exchange: a rank's deltas overflowed the fixed slot; every pipelined kernel no-ops
  // per launch pair: merge entries past the mark regions, by launch parity
  int64_t L_ovf2[2];
  // per bin / import launch
  int64_t np_ovf, ns_ovf, nL_total;
  int64_t ntouched, nmismatch;
  // hot list (argmax): every key with count >= theta is in clist[0..ncl2[cl_act])
  int64_t ncl2[2];
  int32_t cl_act;      // active list counter
  int32_t theta;       // 0 = list not built yet
  int32_t cl_valid;
  int32_t dgen;        // pipelined exchange: iterations begun (launch parity = dgen & 1)
  int64_t cl_measured; // max count found by a measure iteration
  int64_t nskip;       // rebuild iterations so far (stats)
  int64_t nunchecked;  // found-key records beyond the check regions (not verified)
  // posting index: bucket-sorted (key, slot) per region + per-owner logs of the
  // pairs made since its last rebuild (chunks of one pool)
  int32_t post_valid, plog_ovf;
  int64_t pool_used, npost;   // pool chunks handed out since the last rebuild; rebuilds so far
  int64_t nko2[2];            // key records past the fixed slots, by launch parity
  int32_t place_par;          // launch parity of the merge k_place writes out (-1: none)
  int32_t place_nid;          // ... its new token id, merge entries / key records past the fixed slots:
  int64_t place_novf, place_nko;  // k_commit copies them here, so k_place has them in its first round
  int64_t stat_krec, stat_drec, stat_keys;
  int64_t nxovf;  // entries of Dev.xovf (pipelined exchange)  // k_commit work (profiling only): key records, decrement records, keys
  int64_t slot_max;    // pipelined exchange: the largest slot count of the imports since the last poll (every rank)
  // late-merge path (tail.h): per-key posting lists in one pool
  int64_t kpool_used;  // pool entries handed out since the last list build
  int32_t kp_valid;    // 1: the lists hold every live pair (0: rebuild before the next tail launch)
  int32_t tail_exit;   // why the last k_tail stopped: 0 merges done / error, 1 + Sel decision otherwise
  int32_t tail_par;    // launch parity after the last k_tail
  int32_t pad5;
  int64_t mid_nm[2], mid_nh[2];  // mid.h: merged occurrences / new pairs of k_mid_find, by launch parity
  int32_t place_par_prev;        // mid.h: parity of the merge whose new pairs the next find appends (-1: none)
  int32_t pad6;
  // peer exchange (Dev.xw > 0, exchange.h): the producer launch's last workgroup to arrive
  // publishes its record count; the next select launch's import workgroups take every rank's
  // records and the select workgroup waits for them
  int32_t xarr;   // producer workgroups arrived
  int32_t xiarr;  // import workgroups arrived
  int32_t xpend;  // 1: records published and not yet imported
  int32_t xppar;  // their receive-slot parity
  int64_t xpcnt;  // this rank's record count of them
  int32_t xpseq, pad7;
};

// The decision of one k_mark launch (its workgroup 0 writes Sel[parity]; k_apply
// and the host read it).  Every mark workgroup computes the same decision.
constexpr int SEL_MERGE = 0, SEL_SKIP = 1, SEL_DONE = 2, SEL_STALL = 3;  // STALL: mid.h, lists being rebuilt
// IDLE: the run's target merge count is reached -- an iteration the host enqueued past it (so
// that a rebuild iteration inside the batch needs no host round trip to top up) does nothing
constexpr int SEL_IDLE = 4;
struct Sel {
  int32_t decision;
  int32_t skip;       // SKIP_* bits of a rebuild iteration
  int32_t rebuild;    // merge: k_find rebuilds the posting index first (rank-local; the iteration still merges)
  int32_t wown;       // merge: the owner whose posting log holds the winner's new pairs
  int32_t kpn, kpoff; // merge: the winner's per-key posting list (tail.h / mid.h), when built
  int32_t theta_new;  // hot-list rebuild threshold
  int32_t build;      // hot-list counter the rebuild fills
  int32_t W, nid, iter, tag;
  int32_t maxc, ncand, wl, wfp;
  int32_t widL, wg, widR, pad;
  u64 w1, w2;         // content hash of the new token
};

struct LEntry {  // one merge: left token a, right token b, next token c; ya = the new token's length word
  int32_t a, ya, b, c;
};
struct NewPair {
  int32_t target;  // residue whose pk receives the key (-1: none)
  int32_t slot;    // key-table slot
  int32_t len;     // residues of the pair content
  int32_t delta;   // count contribution
  u64 h1, h2;
};
struct DeltaRec {  // 40 bytes, exchanged between ranks
  u64 h1, h2;
  int32_t len, idL, g, idR, delta, pad;
};
static_assert(sizeof(DeltaRec) == 40, "delta record layout");
struct ReplayRec {  // merge replay: the content of trained token K0 + t and one split of it
  u64 h1, h2;
  int32_t len, idL, g, idR;
};
static_assert(sizeof(ReplayRec) == 32, "replay record layout");
struct LogRec {  // one merge of the run (the merge list, device side)
  int32_t nid, count, W, idL, g, idR;
  int64_t nmerged;
};

// a new pair key of a merge, find -> its owner's commit workgroup: content hash,
// representative and n occurrence slots whose pk receive the key (T[tstart ..
// tstart + n), or one slot -(tstart + 1) when tstart < 0)
struct KRec {
  u64 pkey, h1, h2;
  int32_t len, idL, g, idR, n, tstart;
};
static_assert(sizeof(KRec) == 48, "key record layout");

struct Dev {
  // corpus
  int64_t R, nrows;
  int32_t B, B2, B3, pad0;
  const int64_t* row_off;
  int32_t *rsym, *gsym;
  uint16_t* gs16;  // gsym as 16 bits when B^3 + B < 65535 (the merge loop reads these), else null
  // tokens (residue indexed).  tok[s] = {tid, tlen, tprev, pk} of the token
  // starting at slot s (tid -1: not a token start; pk: key id of the pair (this
  // token, the next one), -1: none): one 16-B record, so the scattered reads of a
  // merged occurrence touch one line per neighbour instead of one per field;
  // content hashes come from the vocab (vh1/vh2[tid], L2-resident)
  int4* tok;
  int32_t* pk;    // the bin pass's pair keys (streamed there; k_pack copies them into tok.w)
  int32_t* lab0;  // initial residue labels (= tok[s].x before any merge): the bin pass streams these
  // vocab (token id indexed)
  u64 *vh1, *vh2;
  int32_t* vlen;
  int64_t* voff;  // content of id v = vsym[voff[v] .. voff[v+1])
  int32_t* vsym;
  int64_t KC, VSC;
  // hash powers
  const u64 *pw1, *pw2;
  int64_t pwn;
  // key table
  u64* ht_key;
  int64_t HC;
  int32_t ht_shift, hc_log2;
  // dense keys
  u64 *kh1, *kh2;
  int32_t *klen, *krep, *count, *dcount, *touch, *touched, *scratch;
  int64_t KCAP;     // klist capacity (keys)
  // per-workgroup output regions (no global returning atomics on the hot path)
  int32_t NB;       // grid of the streaming helper kernels
  int32_t NBA;      // find / commit / finalize / bin / import workgroups (one region each)
  int64_t LC;       // merge entries per find region
  int64_t RC;       // new pairs / new keys per commit / bin / import region
  LEntry* L;
  int32_t* Lcnt;
  LEntry* Lovf;
  int64_t Lovf_cap;
  NewPair* np;
  int32_t* npcnt;
  NewPair* npovf;
  int32_t* ns;  // per region workgroup: slots it claimed (listed in klist at region close)
  int32_t* klist;  // every key id (= key-table slot), in claim order; U = reserved length (-1 = unused)
  int64_t* kchunk; // per apply workgroup: [next, end) of its reserved klist chunk
  NewPair* chk;     // per apply workgroup: keys found in the last merge (EHASH check)
  int32_t* chkcnt;
  // posting index: region r = residue slots [r*PR, (r+1)*PR), one per apply workgroup
  int2* post;       // (key, slot) of every live pair at the last rebuild, bucket-sorted per region
  int32_t* poff;    // [NBA][NBKT+1] bucket offsets within a region
  int64_t PR;
  // posting logs: owner j's (key, slot) entries since the rebuild live in pool
  // chunks pch[j * MAXCH + c], c < pnch[j], the last one filled to pfill[j]
  int2* pool;
  int32_t *pch, *pnch, *pfill;
  int64_t POOL_CH;
  int32_t CHUNK, MAXCH;
  // find -> commit records (merge.h)
  KRec* KS;         // [owner][find wg][SK]
  int32_t* cntK;    // [owner][find wg]
  int2* DS;         // [owner][find wg][SD] (key id, count delta)
  int32_t* cntD;
  KRec* KO;         // overflow: key records past their fixed slots
  int64_t KO_cap;
  int2* T;          // [find wg][TC]: {occurrence slot, its key record (KS index)} grouped by new key
  int32_t* Tcnt;    // [find wg]: T entries
  int64_t TC;
  // optional phase timeline (geobpe_debug_timeline): DBG_SLOTS wall-clock stamps per workgroup
  int64_t* dbg;
  int32_t stats, pad4;  // k_commit accumulates stat_* (profiling)
  // pipelined exchange: k_commit writes this rank's delta records straight into the
  // slot buffer (xrec[0 .. xcap), st->ntouched counts them; no touched list, no
  // rank-local delta array, no export pass); null: the touched-list path
  DeltaRec* xrec;
  int64_t xcap;
  // the record counter: null = st->ntouched; the middle regime (mid.h) counts straight
  // into the slot header, which is then final when k_mid_find ends (no header pass)
  int64_t* xcnt;
  int2* xovf;  // (key, delta) of the rare unstaged adds of a pipelined iteration
  // peer exchange (geobpe_comm_peer; exchange.h): every record j < xcapf is also stored straight
  // into rank q's receive area (xpeer[q]: IPC-mapped, over xGMI on a node; this launch's parity
  // half) at the slot of this rank; xrecv = this rank's own area (parity 0).  xw = 0: off
  uint8_t* xpeer[XPEER_MAX];
  uint8_t* xrecv;
  int64_t xslot, xcapf;  // bytes per source slot (XHDR + xcapf records), records per slot
  int32_t xw, xme;       // ranks, this rank
  int32_t xseq, xpar;    // this launch's sequence number and slot parity
  int32_t xloop, xpad;   // loopback rehearsal: this rank is also its own peer (records to its own
                         // slot, imported by content hash; none applied by the producer)
  NewPair* xchk;         // per import workgroup: the keys its import found (not claimed), checked
  int32_t* xchkcnt;      // against their stored content by the next import (EHASH; exchange.h)
  int64_t xchkcap;
  int64_t ovf_cap;
  // late-merge path (tail.h): key d's posting list is kpool[kp_off[d] .. + kp_n[d]) (capacity
  // kp_cap[d]; entries whose token no longer carries the key are skipped); per-merge scratch
  int32_t *kp_off, *kp_n, *kp_cap, *kpool;
  int64_t KPOOL;
  int4* TM;       // merged occurrences {a, ya, b, c}
  int2* TH;       // new pairs {slot, key} (mid.h: two buffers of THcap, by launch parity)
  int4* mcnt;     // mid.h: per find workgroup {TM count, TH count, merged, -} by parity [2][NBA_MAX]
  int32_t* mbk;   // mid.h: per find workgroup, its TH segment's runs by appending workgroup
                  // (bucket k at [mbk[k], mbk[k + 1])), by parity [2][NBA_MAX][MID_APP + 1]
  int4* TS;       // posting entries past a list's capacity {key, position, slot}
  int32_t* TR;    // keys whose list is regrown
  NewPair* TK;    // keys found (not claimed): EHASH check
  int64_t TMcap, THcap;
  int4* ev;       // merge-event log (record mode; see geobpe_set_record_events), or null
  int64_t ev_cap;
  unsigned long long* ev_n;
  // argmax
  int32_t* clist;  // hot list (capacity KCAP)
  LogRec* log;
  State* st;
  Sel* sel;  // [2], by launch parity
};

// ------------------------------------------------------------------ arithmetic
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

// content hash of X ++ [g] ++ Y from the hashes of X and Y and |Y| residues:
// H(s_0..s_{n-1}) = sum (s_i + 1) P^(n-1-i)  mod 2^61-1, two bases
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

// The first error wins (GEOBPE_E*, and where it happened).  Out of line: its call sites sit
// on cold paths of the merge kernels, and inlined, their 64-bit constants were hoisted into
// VGPRs that the 128-VGPR budget of a 1024-thread workgroup then spilled to scratch -- every
// lane of every launch wrote ~28 B of scratch (k_find / k_mid_find: ~7-8 MB of HBM writes
// per launch at the kernel end).  A call materialises them in the cold block instead.
__device__ __attribute__((noinline, cold)) void set_error_at(State* st, int64_t code, int64_t pos) {
  unsigned long long* p = (unsigned long long*)&st->err_code;
  if (atomicCAS(p, 0ULL, (unsigned long long)code) == 0ULL) st->err_pos = pos;
}
__device__ inline void set_error(const Dev& D, int64_t code, int64_t pos) { set_error_at(D.st, code, pos); }

// Python / numpy  (v + 2*pi) % (2*pi)  in float64 (float_rem / npy_divmod)
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

// BPE.get_ind (bpe.py:1164-1189); -1 where the reference raises ValueError
__device__ inline int32_t get_ind(const double* e, int32_t B, double v) {
  int32_t lo = 0, hi = B;  // bisect_right over the B left edges e[0..B-1]
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
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

// ------------------------------------------------------------------ wave / block helpers
__device__ inline int wave_lane() { return threadIdx.x & 63; }

__device__ inline int32_t wave_excl_scan(int32_t v, int32_t& total) {
  int32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(x, o, 64);
    if (wave_lane() >= o) x += y;
  }
  total = __shfl(x, 63, 64);
  return x - v;
}

__device__ inline int32_t wave_sum(int32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ inline int32_t wave_max(int32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide max (all threads get the result); scratch: BLOCK/64 ints
__device__ inline int32_t block_max(int32_t v, int32_t* scratch) {
  v = wave_max(v);
  __syncthreads();
  if (wave_lane() == 0) scratch[threadIdx.x >> 6] = v;
  __syncthreads();
  int32_t r = scratch[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); i++) r = max(r, scratch[i]);
  return r;
}

// block-wide exclusive scan of one int per thread; *total = block sum
// scratch: BLOCK/64 ints
__device__ inline int32_t block_excl_scan(int32_t v, int32_t* total, int32_t* scratch) {
  int32_t wt;
  const int32_t ex = wave_excl_scan(v, wt);
  __syncthreads();
  if (wave_lane() == 0) scratch[threadIdx.x >> 6] = wt;
  __syncthreads();
  int32_t base = 0, tot = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); i++) {
    if (i < (int)(threadIdx.x >> 6)) base += scratch[i];
    tot += scratch[i];
  }
  *total = tot;
  return base + ex;
}

// phase stamp for the debug timeline (no-op unless enabled)
__device__ inline void dbg_stamp(const Dev& D, int k) {
  if (D.dbg && threadIdx.x == 0 && k < DBG_SLOTS) D.dbg[(int64_t)blockIdx.x * DBG_SLOTS + k] = (int64_t)wall_clock64();
}

// debug timeline: a value instead of a time stamp (thread 0)
__device__ inline void dbg_val(const Dev& D, int k, int64_t v) {
  if (D.dbg && threadIdx.x == 0 && k < DBG_SLOTS) D.dbg[(int64_t)blockIdx.x * DBG_SLOTS + k] = v;
}

// key d's stored content equals (h1, h2, len): the three loads issued together and compared
// without short-circuit (`a != x || b != y || ...` loaded them one after another, a round trip each)
__device__ inline bool key_is(const Dev& D, int32_t d, u64 h1, u64 h2, int32_t len) {
  const u64 a = D.kh1[d], b = D.kh2[d];
  const int32_t c = D.klen[d];
  return (a == h1) & (b == h2) & (c == len);
}

__device__ inline uint32_t post_bkt(int32_t d) { return ((uint32_t)d * 2654435761u) >> (32 - NBKT_LOG2); }

// token record fields (int4 tok[s] = {tid, tlen, tprev, pk})
__device__ inline int32_t* tok_f(const Dev& D, int64_t s, int f) { return reinterpret_cast<int32_t*>(D.tok + s) + f; }
__device__ inline int32_t tok_pk(const Dev& D, int64_t s) { return D.tok[s].w; }
// tok.y = residues (low 16 bits) | junction symbol after the token (high 16 bits,
// 0xFFFF = chain end; only when the 16-bit symbols exist, else 0)
__device__ inline int32_t tok_len(int32_t y) { return y & 0xFFFF; }
// the junction symbol after a token whose length word is y and last residue e
__device__ inline int32_t next_glue(const Dev& D, int32_t y, int64_t e) {
  if (D.gs16) {
    const uint32_t v = (uint32_t)y >> 16;
    return v == 0xFFFF ? -1 : (int32_t)v;
  }
  return D.gsym[e];
}
// junction symbol after residue i (16-bit copy when B^3 fits, else the int32 array)
__device__ inline int32_t glue(const Dev& D, int64_t i) {
  if (D.gs16) {
    const uint16_t v = D.gs16[i];
    return v == 0xFFFF ? -1 : (int32_t)v;
  }
  return D.gsym[i];
}

__device__ inline uint16_t key_fp(int32_t d) { return (uint16_t)((uint32_t)d % 65535u); }

// a key whose rank-local delta left 0 joins the touched list: one reservation per
// wave instruction (the lanes calling this are exactly the active ones)
__device__ inline void touched_append(const Dev& D, int32_t d) {
  const u64 m = __ballot(1);
  const int lane = wave_lane();
  const int leader = __ffsll((long long)m) - 1;
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd((unsigned long long*)&D.st->ntouched, (unsigned long long)__popcll(m));
  base = __shfl(base, leader, 64);
  const unsigned long long j = base + __popcll(m & ((1ULL << lane) - 1));
  if ((int64_t)j < D.KCAP)
    D.touched[j] = d;
  else
    set_error(D, GEOBPE_ECAPACITY, -31);
}

// count update target: global counts, or the rank-local delta + touched list.
// A key joins the touched list when its delta leaves 0 (the add that returns 0);
// a key whose delta came back to 0 and left again is listed twice -- the export
// takes each delta with an exchange, so the later copy carries 0 and the import
// skips it.  No per-key epoch table, no returning exchange on a second array.
__device__ inline void global_add(const Dev& D, int32_t d, int32_t v, bool to_delta) {
  if (!to_delta) {
    atomicAdd(&D.count[d], v);
    return;
  }
  if (D.xrec) {  // pipelined exchange, k_find's rare path: (key, delta) to a side list that
                 // k_commit turns into records (a record built here costs k_find its register budget)
    const unsigned long long j = atomicAdd((unsigned long long*)&D.st->nxovf, 1ULL);
    if ((int64_t)j < D.KCAP)
      D.xovf[j] = make_int2(d, v);
    else
      set_error(D, GEOBPE_ECAPACITY, -32);
    return;
  }
  if (atomicAdd(&D.dcount[d], v) == 0) touched_append(D, d);
}

// delta record j of this rank: its local list (xrec: what a stalled merge's full re-exchange
// reads) and, with the peer exchange, rank q's receive slot of this rank for every other q --
// direct stores into the peer's memory, no collective (j < xcapf; a count past it stalls the
// pipeline on every rank and the merge is re-exchanged in full)
__device__ __attribute__((always_inline)) inline void x_put_rec(const Dev& D, int64_t j, const DeltaRec& r, int32_t err) {
  if (j >= D.xcap) {
    set_error(D, GEOBPE_ECAPACITY, err);
    return;
  }
  D.xrec[j] = r;
  if (D.xw > 0 && !D.xloop && r.pad > 0 && r.delta != 0) {
    // the peer exchange applies this rank's own change here, where the record is made (the
    // import takes only the other ranks'); nothing in a producer launch reads the counts, so
    // this is the import's add moved earlier.  A theta crossing joins the hot list directly.
    const int32_t d = r.pad - 1;
    const int32_t old = atomicAdd(&D.count[d], r.delta);
    const int32_t th = D.st->theta;
    if (r.delta > 0 && th > 0 && old < th && old + r.delta >= th) {
      const int64_t k = (int64_t)atomicAdd((unsigned long long*)&D.st->ncl2[D.st->cl_act], 1ULL);
      if (k < D.KCAP)
        D.clist[k] = d;
      else
        D.st->cl_valid = 0;
    }
  }
  if ((D.xw > 1 || D.xloop) && j < D.xcapf) {
    const unsigned long long* v = reinterpret_cast<const unsigned long long*>(&r);
#pragma unroll
    for (int q = 0; q < XPEER_MAX; q++) {  // (static indices: a runtime index into the kernel-argument
      if (q >= D.xw || (q == D.xme && !D.xloop)) continue;  // array copies the whole Dev to scratch)
      // written through to the peer's memory (system-scope stores: no dirty line left in this
      // XCD's L2, so the producer's end needs no L2 write-back before the header)
      unsigned long long* o =
          reinterpret_cast<unsigned long long*>(reinterpret_cast<DeltaRec*>(D.xpeer[q] + (int64_t)D.xme * D.xslot + XHDR) + j);
#pragma unroll
      for (int i = 0; i < 5; i++) __hip_atomic_store(o + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// pipelined exchange, k_commit's rare unstaged adds: a delta record straight into the
// rank's slot (one reservation per wave instruction on the record counter)
__device__ inline void rec_add(const Dev& D, int32_t d, int32_t v) {
  const u64 m = __ballot(1);
  const int lane = wave_lane();
  const int leader = __ffsll((long long)m) - 1;
  unsigned long long base = 0;
  if (lane == leader)
    base = atomicAdd((unsigned long long*)(D.xcnt ? D.xcnt : &D.st->ntouched), (unsigned long long)__popcll(m));
  base = __shfl(base, leader, 64);
  const int64_t j = (int64_t)(base + __popcll(m & ((1ULL << lane) - 1)));
  DeltaRec r;
  r.h1 = D.kh1[d];
  r.h2 = D.kh2[d];
  r.len = D.klen[d];
  r.idL = D.krep[3 * (int64_t)d];
  r.g = D.krep[3 * (int64_t)d + 1];
  r.idR = D.krep[3 * (int64_t)d + 2];
  r.delta = v;
  r.pad = d + 1;
  x_put_rec(D, j, r, -33);
}

// rank-local deltas of one workgroup whose keys join the touched list: buffered in
// LDS, one reservation on the global list per workgroup (a wave-level reservation
// from every workgroup queues thousands of atomics on one counter)
constexpr int TB_N = 2048;
struct TouchBuf {
  int32_t n;
  int32_t buf[TB_N];
};
__device__ inline void touch_add(const Dev& D, TouchBuf& tb, int32_t d, int32_t v) {
  if (atomicAdd(&D.dcount[d], v) != 0) return;
  const int32_t j = atomicAdd(&tb.n, 1);
  if (j < TB_N)
    tb.buf[j] = d;
  else
    touched_append(D, d);
}
__device__ inline void touch_flush(const Dev& D, TouchBuf& tb) {
  __shared__ unsigned long long s_base;
  __syncthreads();
  const int32_t n = min(tb.n, TB_N);
  if (threadIdx.x == 0 && n > 0) s_base = atomicAdd((unsigned long long*)&D.st->ntouched, (unsigned long long)n);
  __syncthreads();
  for (int32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const int64_t j = (int64_t)s_base + i;
    if (j < D.KCAP)
      D.touched[j] = tb.buf[i];
    else
      set_error(D, GEOBPE_ECAPACITY, -31);
  }
}

// LDS-staged per-workgroup partial counts, flushed with one global atomic per
// distinct key per workgroup (open addressing, 8 probes, then straight to global)
template <int LOG2>
struct AggT {
  static constexpr int N = 1 << LOG2;
  int32_t key[N];
  int32_t val[N];
  __device__ static uint32_t slot(int32_t d) { return ((uint32_t)d * 2654435761u) >> (32 - LOG2); }
};
using Agg = AggT<9>;      // 4 KB: recount
using AggBig = AggT<13>;  // 64 KB: bin / merge-apply / import (early merges touch ~10^4 keys per workgroup)

template <class A>
__device__ inline void agg_init(A& s) {
  for (int i = threadIdx.x; i < A::N; i += blockDim.x) {
    s.key[i] = -1;
    s.val[i] = 0;
  }
  __syncthreads();
}
// true if staged in LDS
template <class A>
__device__ inline bool agg_stage(A& s, int32_t d, int32_t v) {
  uint32_t h = A::slot(d);
#pragma unroll 1
  for (int probe = 0; probe < 8; probe++) {
    const int32_t k = s.key[h];
    if (k == d) {
      atomicAdd(&s.val[h], v);
      return true;
    }
    if (k == -1) {
      const int32_t old = atomicCAS(&s.key[h], -1, d);
      if (old == -1 || old == d) {
        atomicAdd(&s.val[h], v);
        return true;
      }
    }
    h = (h + 1) & (A::N - 1);
  }
  return false;
}
template <class A>
__device__ inline void agg_add(A& s, const Dev& D, int32_t d, int32_t v, bool to_delta) {
  if (!agg_stage(s, d, v)) global_add(D, d, v, to_delta);
}
template <class A>
__device__ inline void agg_flush(A& s, const Dev& D, bool to_delta) {
  __syncthreads();
  for (int i = threadIdx.x; i < A::N; i += blockDim.x) {
    const int32_t k = s.key[i];
    if (k >= 0 && s.val[i] != 0) global_add(D, k, s.val[i], to_delta);
  }
}

// hot-list appends (argmax): a key whose count crosses theta from below joins
// clist; LDS-buffered, one global reservation per workgroup
constexpr int HOT_BUF = 256;
struct HotApp {
  int32_t n;
  int32_t buf[HOT_BUF];
};
__device__ inline void hot_init(HotApp& h) {
  if (threadIdx.x == 0) h.n = 0;
}
__device__ inline void hot_store(const Dev& D, int64_t k, int32_t d) {
  if (k < D.KCAP)
    D.clist[k] = d;
  else
    D.st->cl_valid = 0;  // list lost an entry: the next k_mark has it rebuilt
}
__device__ inline void hot_push(const Dev& D, HotApp& h, int32_t d) {
  const int32_t j = atomicAdd(&h.n, 1);
  if (j < HOT_BUF)
    h.buf[j] = d;
  else
    hot_store(D, (int64_t)atomicAdd((unsigned long long*)&D.st->ncl2[D.st->cl_act], 1ULL), d);
}
__device__ inline void hot_flush(const Dev& D, HotApp& h) {
  __shared__ int64_t s_base;
  __syncthreads();
  const int32_t n = min(h.n, HOT_BUF);
  if (threadIdx.x == 0 && n > 0)
    s_base = (int64_t)atomicAdd((unsigned long long*)&D.st->ncl2[D.st->cl_act], (unsigned long long)n);
  __syncthreads();
  for (int32_t i = threadIdx.x; i < n; i += blockDim.x) hot_store(D, s_base + i, h.buf[i]);
}
// global count update with the theta-crossing check (positive deltas only can cross)
__device__ inline void count_add_hot(const Dev& D, HotApp& h, int32_t d, int32_t v, int32_t th) {
  if (v > 0 && th > 0) {
    const int32_t old = atomicAdd(&D.count[d], v);
    if (old < th && old + v >= th) hot_push(D, h, d);
  } else {
    atomicAdd(&D.count[d], v);
  }
}
template <class A>
__device__ inline void agg_add_hot(A& s, const Dev& D, HotApp& h, int32_t d, int32_t v, bool to_delta, int32_t th) {
  if (agg_stage(s, d, v)) return;
  if (to_delta)
    global_add(D, d, v, true);
  else
    count_add_hot(D, h, d, v, th);
}
template <class A>
__device__ inline void agg_flush_hot(A& s, const Dev& D, HotApp& h, bool to_delta, int32_t th) {
  __syncthreads();
  if (to_delta) {
    // all of a thread's returning adds in flight together; the keys whose delta
    // left 0 join the touched list with ONE reservation per workgroup (a single
    // global counter serialises at the memory side: one add per wave cost ~70 us)
    constexpr int U = A::N / 1024 > 0 ? A::N / 1024 : 1;  // slots per thread at 1024 threads
    __shared__ int32_t s_red_t[32];
    __shared__ unsigned long long s_base_t;
    int32_t k[U];
    int32_t nt = 0;
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int i = threadIdx.x + u * (int)blockDim.x;
      k[u] = i < A::N ? s.key[i] : -1;
      const int32_t v = k[u] >= 0 ? s.val[i] : 0;
      if (v == 0) k[u] = -1;
      const int32_t old = k[u] >= 0 ? atomicAdd(&D.dcount[k[u]], v) : 1;
      if (old != 0) k[u] = -1;
      nt += k[u] >= 0;
    }
    for (int i = threadIdx.x + U * (int)blockDim.x; i < A::N; i += blockDim.x) {  // blockDim < 1024
      const int32_t kk = s.key[i];
      if (kk >= 0 && s.val[i] != 0) global_add(D, kk, s.val[i], true);
    }
    int32_t tot;
    const int32_t ex = block_excl_scan(nt, &tot, s_red_t);
    if (threadIdx.x == 0)
      s_base_t = tot ? atomicAdd((unsigned long long*)&D.st->ntouched, (unsigned long long)tot) : 0ULL;
    __syncthreads();
    int64_t j = (int64_t)s_base_t + ex;
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (k[u] < 0) continue;
      if (j < D.KCAP)
        D.touched[j] = k[u];
      else
        set_error(D, GEOBPE_ECAPACITY, -31);
      j++;
    }
  } else {
    // every slot's add in flight before the first result is needed: the returning
    // adds (positive deltas: the theta-crossing check) of a thread are issued back
    // to back, not one round trip per slot
    constexpr int U = A::N / 1024 > 0 ? A::N / 1024 : 1;
    int32_t k[U], v[U], old[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int i = threadIdx.x + u * (int)blockDim.x;
      k[u] = i < A::N ? s.key[i] : -1;
      v[u] = k[u] >= 0 ? s.val[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      old[u] = 0;
      if (v[u] > 0 && th > 0)
        old[u] = atomicAdd(&D.count[k[u]], v[u]);
      else if (v[u] != 0)
        atomicAdd(&D.count[k[u]], v[u]);
    }
    dbg_stamp(D, 34);
#pragma unroll
    for (int u = 0; u < U; u++)
      if (v[u] > 0 && th > 0 && old[u] < th && old[u] + v[u] >= th) hot_push(D, h, k[u]);
    dbg_stamp(D, 35);
    for (int i = threadIdx.x + U * (int)blockDim.x; i < A::N; i += blockDim.x) {  // blockDim < 1024
      const int32_t kk = s.key[i];
      if (kk >= 0 && s.val[i] != 0) count_add_hot(D, h, kk, s.val[i], th);
    }
  }
  hot_flush(D, h);
  dbg_stamp(D, 36);
}


// key-table probing: the first slot of a key and, given the value already read
// there, find-or-claim (CAS) its slot; *claimed = true if this thread inserted it
__device__ inline u64 ht_first_slot(const Dev& D, u64 k) { return (k * 0xD6E8FEB86659FD93ULL) >> D.ht_shift; }

// a key-table probe that sees claims other workgroups made during this launch
// (agent scope: skips this CU's stale L1), so late arrivals find the key instead
// of queueing a CAS on the same slot
__device__ inline u64 ht_probe(const Dev& D, u64 s) {
  return __hip_atomic_load(&D.ht_key[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ inline int32_t ht_resolve(const Dev& D, u64 k, u64 s, u64 cur, bool* claimed) {
  const u64 mask = (u64)D.HC - 1;
  *claimed = false;
  // keep cur an opaque register value: otherwise the loop's phi of (cur, table
  // load) can be folded into a load through a phi of pointers -- a flat load
  // via the scratch stack when cur came from a caller's struct
  asm volatile("" : "+v"(cur));
  for (int64_t probe = 0; probe < D.HC; probe++) {
    if (cur == k) return (int32_t)s;
    if (cur == 0) {
      const u64 old = atomicCAS((unsigned long long*)&D.ht_key[s], 0ULL, (unsigned long long)k);
      if (old == 0) {
        *claimed = true;
        return (int32_t)s;
      }
      if (old == k) return (int32_t)s;
    }
    s = (s + 1) & mask;
    cur = ht_probe(D, s);
  }
  set_error(D, GEOBPE_ECAPACITY, -2);
  return -1;
}

// the commit workgroup that owns a key-table slot / a key (by its first probe slot)
__device__ inline int owner_of_slot(const Dev& D, u64 s) { return (int)((s * (u64)D.NBA) >> D.hc_log2); }
__device__ inline int owner_of_key(const Dev& D, u64 pkey) { return owner_of_slot(D, ht_first_slot(D, pkey)); }

__device__ inline int32_t ht_insert(const Dev& D, u64 h1, u64 h2, int32_t len, bool* claimed) {
  const u64 k = probe_key(h1, h2, len);
  const u64 s = ht_first_slot(D, k);
  return ht_resolve(D, k, s, ht_probe(D, s), claimed);
}

// hash of X ++ [g] ++ Y with the powers P^(|Y|syms+1), P^|Y|syms given
__device__ inline void combine_pw(u64 x1, u64 x2, int32_t g, u64 y1, u64 y2, u64 p1a, u64 p1b, u64 p2a, u64 p2b,
                                  u64& o1, u64& o2) {
  const u64 gg = (u64)(g + 1);
  o1 = addmod61(addmod61(mulmod61(x1, p1a), mulmod61(gg, p1b)), y1);
  o2 = addmod61(addmod61(mulmod61(x2, p2a), mulmod61(gg, p2b)), y2);
}

}  // namespace gb
