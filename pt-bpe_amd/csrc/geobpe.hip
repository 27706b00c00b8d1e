// geobpe.hip -- MI355X (gfx950) GeoBPE merge loop: host side of the C-ABI
// declared in include/geobpe.h.  Kernels: kernels.h; device layout: device.h.
//
// Replaces the Python/dict hot path of foldingdiff/bpe.py (BPE.initialize /
// bin / step / quantize).  Integer work only (no
// MFMA).  One merge iteration is four stream-ordered launches with no host
// synchronisation:
//   k_select  one 1024-thread workgroup: hot-list argmax + reference key-string
//             tie-break (wave-parallel comparisons on LDS copies of the tied keys),
//             the decision record (Sel) and merge-log entry
//   k_find    the winner's occurrences (posting index), greedy run walks, the new
//             neighbour keys grouped per owner workgroup (merge.h)
//   k_commit  per owner: one key-table resolve and one count update per key,
//             posting-log space; hot-list rebuild iterations
//   k_place   per region: token rewrites, pk of the occurrences, posting-log entries
// The bin pass is k_pairs_all + k_finalize.

#include <dlfcn.h>
#include <hip/hip_ext.h>
#include <rccl/rccl.h>  // types only: the functions are resolved at run time (the process's RCCL)

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "device.h"
#include "keyjson.h"
#include "kernels.h"
#include "featurize.h"
#include "rmsd.h"
#include "glue.h"

using namespace gb;

// RCCL entry points, resolved with dlsym from the RCCL library the process already uses
// (PyTorch's: one RCCL instance per process)
struct RcclApi {
  void* h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

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
  std::vector<void*> allocs;
  State* h_state = nullptr;  // pinned mirror
  Sel* h_sel = nullptr;      // pinned copy of the last decision (step_select)
  LogRec* h_log = nullptr;   // pinned mirror of the merge log, pulled by geobpe_run_log
  int64_t h_log_cap = 0;
  bool keys_ready = false;
  bool distributed = false;
  bool bin_dense = true;
  // merge replay (geobpe_replay_load): the trained tokens K0.. as forced merges
  ReplayRec* replay = nullptr;
  int64_t replay_n = 0;
  // merge-event log (geobpe_set_record_events): int4 {merge, left start, right start, 0}
  int4* ev = nullptr;
  int64_t ev_cap = 0;
  unsigned long long* ev_n = nullptr;
  int32_t bin_cube[2] = {0, 0};  // cube shape (CL, CG) of the last dense bin
  int64_t global_residues = 0;
  int32_t rank = 0;  // this context's slot in the pipelined exchange
  // host vocab mirror (content per token id), synced lazily from the device log
  std::vector<std::vector<int32_t>> vocab;
  int32_t K0 = 0;
  int ncu = 256;
  int nb = 2048;  // grid of the streaming helper kernels (= D.NB)
  int64_t gen = 0;            // merge-loop launch pairs so far (parity selects Sel / overflow buffers)
  bool mark_pending = false;  // step_select decided a merge whose mark/apply are due
  bool place_pending = false; // a k_commit ran whose k_place has not (it rides with the next k_select)
  bool pipelined = false;     // between geobpe_pipeline_begin and _end (device-side parity)
  int nba = 256;  // find / commit / finalize / bin / import workgroups (= D.NBA, <= NBA_MAX)
  // late-merge path (tail.h): merges whose count is <= tail_thresh run in k_tail
  int64_t tail_thresh = 0;     // 0: never (the mid path is faster at every count measured on C3)
  bool tail_on = false;        // switched (one way: the full-grid kernels' posting index goes stale)
  bool tail_ready = false;     // its arrays are allocated
  int64_t hold_us = 0;         // geobpe_set_hold: a k_hold launch before each batch of iterations
  // run_batches: iterations past a batch's target idle on the device (SEL_IDLE), so a rebuild
  // iteration inside the batch costs no host round trip; run_end = target merges + 1 (0: off)
  int32_t run_end = 0;
  int spec = 1;                // iterations enqueued past the run's last batch target (GEOBPE_SPEC)
  double decay = 0;            // maxc ratio per merge over the last pulled batch (0: unknown)
  // middle regime (mid.h): merges whose count is <= mid_thresh run as k_mid_sel + k_mid_find
  int64_t mid_thresh = 65536;  // 0: never (C3 merges 11..1000, round 5 kernels: 32768 -> 32.2k, 49152 -> 32.6k, 65536 -> 32.8k, 98304 -> 32.8k merges/s)
  bool mid_on = false;         // switched (one way)
  bool place_mid = false;      // the pending place is k_mid_sel's (else k_place's)
  // the multi-rank exchange owned by the engine (geobpe_comm_*, geobpe_run_exchange)
  int x_kind = 0;  // 0: none, 1: RCCL communicator, 2: host callback
  RcclApi rccl;
  ncclComm_t comm = nullptr;
  geobpe_allgather_fn x_fn = nullptr;
  void* x_user = nullptr;
  int32_t x_world = 1, x_rank = 0;
  uint8_t *x_pbuf = nullptr, *x_gath = nullptr, *x_tmp = nullptr, *x_flat = nullptr;
  int64_t* x_head = nullptr;  // the slot header of the last pipelined iteration (its record count)
  int64_t x_pcap = 0, x_tmp_bytes = 0, x_flat_bytes = 0, x_gath_bytes = 0;
  uint8_t *x_hsend = nullptr, *x_hrecv = nullptr;  // (host callback: pinned staging)
  int64_t x_hbytes = 0;
  int64_t x_ahead = 1, x_capf = 1024, x_fixed = 0;  // poll window and slot size carry over between runs
  // peer exchange (exchange.h; geobpe_comm_peer): this rank's receive area (2 parities x
  // x_world slots), every rank's area as mapped here (IPC handles; [x_rank] = x_recv), the
  // host's count of producer launches (each launch's sequence number, the same on every rank)
  bool x_peer_want = true, x_peer_ready = false, x_pending = false, x_cpwait = true, x_loop = false;
  uint8_t* x_recv = nullptr;
  uint8_t* x_peers[XPEER_MAX] = {};
  int64_t x_slot = 0, x_rcapf = 0;
  int64_t x_hseq = 1, x_prev_seq = 0;
  LogRec* x_hlog = nullptr;  // (pinned: a batch's merge records, pulled with its poll)
  int32_t* x_hbeg = nullptr; // (pinned: dgen / stall for a pipeline begin without a synchronisation)
  int64_t enq = 0, enq_synced = -1;  // merge iterations enqueued; the count at the last state sync
  double x_decay = 0;        // the winner count's decay per merge over the last batch (0: unknown)
  LogRec x_last{};           // the last merge's record seen by an exchange run's poll, and its index
  int64_t x_last_i = -1;
  NewPair* x_chk = nullptr;  // the imports' found keys, checked by the next import (exchange.h)
  int32_t* x_chkcnt = nullptr;
  int64_t x_chkcap = 0;
  int64_t x_collapse_at = 32768;  // the sharded loop collapses below this count (GEOBPE_COLLAPSE_AT)
  int64_t x_shards = 1;           // a world-1 rehearsal of one rank's share of an N-way run (GEOBPE_XSHARDS = N): N's thresholds
  // collapse at the middle-regime switch (geobpe_set_collapse): every rank then holds the whole
  // corpus and runs the one-rank loop; its own rows are [own_row0, own_row1) of it
  bool collapse_on = true, collapsed = false;
  // x_collapse_prepare: every rank's sizes and bases, the gathered junction symbols and row offsets
  bool cg_ready = false;
  std::vector<int64_t> cg_nR, cg_nN, cg_bR, cg_bN, cg_rows;
  int64_t cg_Lmax = 1;
  int32_t* cg_gsym = nullptr;
  uint16_t* cg_gs16 = nullptr;
  int64_t* cg_row = nullptr;
  int64_t own_row0 = 0, own_row1 = -1;
  // profiling
  bool prof = false;
  int prof_stride = 1;      // time every prof_stride-th launch of each kernel
  std::string prof_filter;  // ",name,name," or empty = every kernel
  std::map<std::string, int64_t> prof_seen;
  std::map<std::string, std::pair<double, int64_t>> ktime;
  struct Pend {
    std::string name;
    hipEvent_t a, b;
  };
  std::vector<Pend> pending;
  std::vector<hipEvent_t> evpool, evall;
};

namespace {

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
int dalloc(geobpe_ctx* c, T** p, int64_t n, int fill = -1) {
  if (n <= 0) n = 1;
  void* q = nullptr;
  hipError_t e = hipMalloc(&q, (size_t)n * sizeof(T));
  if (e != hipSuccess)
    return fail(c, GEOBPE_EHIP, "hipMalloc(%lld bytes): %s", (long long)(n * sizeof(T)), hipGetErrorString(e));
  c->allocs.push_back(q);
  *p = (T*)q;
  if (fill >= 0) {
    e = hipMemsetAsync(q, fill, (size_t)n * sizeof(T), c->stream);
    if (e != hipSuccess) return fail(c, GEOBPE_EHIP, "hipMemsetAsync: %s", hipGetErrorString(e));
  }
  return 0;
}

template <class T>
void dfree(geobpe_ctx* c, T** p) {
  if (!*p) return;
  auto it = std::find(c->allocs.begin(), c->allocs.end(), (void*)*p);
  if (it != c->allocs.end()) c->allocs.erase(it);
  hipFree((void*)*p);
  *p = nullptr;
}

// ---------------------------------------------------------------- light kernel timing
// timing-only events: no system-scope fence (an L2 writeback + invalidate) when one
// completes -- with it, each sampled launch opened a 7-20 us gap in the merge loop
// (GEOBPE_EVENT_FENCE=1: the default events, A/B)
hipEvent_t make_event(geobpe_ctx* c) {
  static const bool fence = getenv("GEOBPE_EVENT_FENCE") && atoi(getenv("GEOBPE_EVENT_FENCE")) == 1;
  hipEvent_t e;
  if (fence)
    hipEventCreate(&e);
  else
    hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
  c->evall.push_back(e);
  return e;
}
hipEvent_t take_event(geobpe_ctx* c) {
  if (c->evpool.empty()) return make_event(c);
  hipEvent_t e = c->evpool.back();
  c->evpool.pop_back();
  return e;
}

// HIP events recorded on the context stream around a launch; collected (one
// synchronize) only when geobpe_kernel_ms() is called
struct Timed {
  geobpe_ctx* c;
  const char* name;
  hipEvent_t a = nullptr, b = nullptr;
  Timed(geobpe_ctx* c_, const char* n) : c(c_), name(n) {
    if (!c->prof) return;
    if (!c->prof_filter.empty() && c->prof_filter.find("," + std::string(n) + ",") == std::string::npos) return;
    if (c->prof_stride > 1 && (c->prof_seen[n]++ % c->prof_stride) != 0) return;
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

// a sampled single-kernel launch of the merge loop: the start / stop stamps ride on the kernel's
// own dispatch packet (hipExtLaunchKernelGGL) -- no marker packets in the stream, where a pair
// of hipEventRecord around the launch opened an 8-15 us gap before it (profiles/r4_final/)
bool sample_events(geobpe_ctx* c, const char* n, hipEvent_t* a, hipEvent_t* b) {
  if (!c->prof) return false;
  if (!c->prof_filter.empty() && c->prof_filter.find("," + std::string(n) + ",") == std::string::npos) return false;
  // (the middle launch of every stride: a run's first launch of a kernel starts cold)
  if (c->prof_stride > 1 && (c->prof_seen[n]++ % c->prof_stride) != c->prof_stride / 2) return false;
  *a = take_event(c);
  *b = take_event(c);
  c->pending.push_back({n, *a, *b});
  return true;
}
#define LAUNCH_T(c, name, kernel, grid, block, shmem, ...)                                         \
  do {                                                                                           \
    hipEvent_t ea_ = nullptr, eb_ = nullptr;                                                     \
    if (sample_events((c), (name), &ea_, &eb_))                                                  \
      hipExtLaunchKernelGGL(kernel, grid, block, shmem, (c)->stream, ea_, eb_, 0, __VA_ARGS__); \
    else                                                                                         \
      hipLaunchKernelGGL(kernel, grid, block, shmem, (c)->stream, __VA_ARGS__);                  \
  } while (0)

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

// ---------------------------------------------------------------- state helpers
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
    case GEOBPE_ESTATE:
      return fail(c, GEOBPE_ESTATE, "inconsistent token links at slot %lld (internal error)", (long long)pos);
    default:
      return fail(c, (int)code, "device error %lld at %lld", (long long)code, (long long)pos);
  }
}

// the last committed merge's k_place (or mid.h place), when no select launch has carried it yet
void flush_place(geobpe_ctx* c) {
  if (!c->place_pending) return;
  c->place_pending = false;
  Timed t(c, "place");
  if (c->place_mid) {  // token rewrites, then the posting entries, then nothing is pending
    hipLaunchKernelGGL(k_mid_sel, dim3(1 + c->nba), dim3(ABLOCK), 0, c->stream, c->D, INT32_MIN, 0, 0);
    hipLaunchKernelGGL(k_mid_find<false>, dim3(MID_APP), dim3(ABLOCK), 0, c->stream, c->D, (int)(c->gen & 1), 0, 0);
    hipLaunchKernelGGL(k_mid_flushed, dim3(1), dim3(64), 0, c->stream, c->D);
  } else {
    hipLaunchKernelGGL(k_place, dim3(c->nba), dim3(ABLOCK), 0, c->stream, c->D);
  }
}

int sync_state(geobpe_ctx* c) {
  flush_place(c);
  HIPCHK(c, hipMemcpyAsync(c->h_state, c->D.st, sizeof(State), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->enq_synced = c->enq;  // (h_state holds the state after every iteration enqueued so far)
  return check_device_error(c);
}

// zero the overflow / new-key counters before a bin() or an import chunk
int reset_region_counters(geobpe_ctx* c) {
  HIPCHK(c, hipMemsetAsync(&c->D.st->np_ovf, 0, 3 * sizeof(int64_t), c->stream));
  return 0;
}

// pull the device merge log into the host vocab mirror
int sync_vocab(geobpe_ctx* c) {
  int rc;
  if ((rc = sync_state(c))) return rc;
  const int64_t have = (int64_t)c->vocab.size(), K = c->h_state->K;
  if (K <= have) return 0;
  std::vector<LogRec> lr(K - have);
  HIPCHK(c, hipMemcpy(lr.data(), c->D.log + (have - c->K0), lr.size() * sizeof(LogRec), hipMemcpyDeviceToHost));
  for (const LogRec& r : lr) {
    if (r.nid != (int32_t)c->vocab.size()) return fail(c, GEOBPE_EARG, "merge log out of order");
    std::vector<int32_t> x(c->vocab[r.idL]);
    x.push_back(r.g);
    x.insert(x.end(), c->vocab[r.idR].begin(), c->vocab[r.idR].end());
    c->vocab.push_back(std::move(x));
  }
  return 0;
}

int alloc_keys(geobpe_ctx* c) {
  if (c->keys_ready) return 0;
  Dev& D = c->D;
  const int64_t base = c->distributed && c->global_residues > c->R ? c->global_residues : c->R;
  D.KCAP = 3 * base + 65536 + (int64_t)c->nba * KL_CHUNK;  // bin pairs + 2 new pairs per merge + chunk tails
  int64_t hc = 1 << 16;
  while (hc < 2 * D.KCAP) hc <<= 1;
  D.HC = hc;
  int sh = 0;
  while ((1LL << sh) < hc) sh++;
  D.ht_shift = 64 - sh;
  D.hc_log2 = sh;
  int rc;
  // key arrays are indexed by the key id = key-table slot
  if ((rc = dalloc(c, &D.ht_key, D.HC, 0)) || (rc = dalloc(c, &D.kh1, D.HC)) || (rc = dalloc(c, &D.kh2, D.HC)) ||
      (rc = dalloc(c, &D.klen, D.HC)) || (rc = dalloc(c, &D.krep, 3 * D.HC, 0xFF)) ||
      (rc = dalloc(c, &D.count, D.HC + 16, 0)) || (rc = dalloc(c, &D.scratch, D.HC + 16, 0)) ||
      (rc = dalloc(c, &D.klist, D.KCAP, 0xFF)) || (rc = dalloc(c, &D.kchunk, 2 * (int64_t)c->nba, 0)))
    return rc;
  if (c->distributed) {
    if ((rc = dalloc(c, &D.xovf, D.KCAP)) || (rc = dalloc(c, &D.dcount, D.HC, 0)) ||
        (rc = dalloc(c, &D.touched, D.KCAP)))
      return rc;
  }
  if ((rc = dalloc(c, &D.clist, D.KCAP))) return rc;
  c->keys_ready = true;
  return 0;
}

// after the bin pass: pair keys into the token records, 16-bit junction symbols
void enqueue_pack(geobpe_ctx* c) {
  Timed t(c, "bin_pack");
  hipLaunchKernelGGL(k_pack, dim3(c->nb), dim3(BLOCK), 0, c->stream, c->D);
}

// the launches of one merge iteration (no host synchronisation)
void enqueue_commit(geobpe_ctx* c, bool to_delta) {
  Timed t(c, "finalize");
  hipLaunchKernelGGL(k_finalize, dim3(c->nba), dim3(ABLOCK), 0, c->stream, c->D, to_delta ? 1 : 0);
}

// one merge iteration = k_select (argmax, decision) -> k_mark (occurrences) ->
// k_apply, on launch parity gen & 1 (the double-buffered Sel record and
// merge-overflow counter)
void enqueue_select(geobpe_ctx* c) {
  c->enq++;
  if (c->replay) {
    flush_place(c);
    Timed t(c, "select");
    hipLaunchKernelGGL(k_select_replay, dim3(1), dim3(64), 0, c->stream, c->D, (int)(c->gen & 1),
                       (const ReplayRec*)c->replay, c->replay_n);
    return;
  }
  if (c->place_pending && c->place_mid) flush_place(c);
  const int grid = c->place_pending ? 1 + c->nba : 1;  // (+ the previous merge's k_place in workgroups 1..nba)
  c->place_pending = false;
  LAUNCH_T(c, "select", k_select, dim3(grid), dim3(SBLOCK), 0, c->D, (int)(c->gen & 1), c->run_end, grid > 1 ? 1 : 0, 0);
}
void enqueue_mark(geobpe_ctx* c) {
  LAUNCH_T(c, "find", k_find, dim3(c->nba), dim3(ABLOCK), 0, c->D, c->distributed ? 1 : 0, (int)(c->gen & 1));
}
void enqueue_apply(geobpe_ctx* c) {
  LAUNCH_T(c, "commit", k_commit<false>, dim3(c->nba), dim3(ABLOCK), 0, c->D, c->distributed ? 1 : 0, (int)(c->gen & 1));
  c->place_pending = true;
  c->place_mid = false;
  if (c->ev)
    hipLaunchKernelGGL(k_events, dim3(c->nba), dim3(BLOCK), 0, c->stream, c->D, (int)(c->gen & 1), c->ev, c->ev_cap,
                       c->ev_n);
  c->gen++;
}
void enqueue_iteration(geobpe_ctx* c) {
  enqueue_select(c);
  enqueue_mark(c);
  enqueue_apply(c);
}

// one merge iteration of the middle regime (mid.h): select (+ the previous place) -> find
void enqueue_iteration_mid(geobpe_ctx* c) {
  c->enq++;
  const int par = (int)(c->gen & 1);
  {
    const bool carry = c->place_pending && c->place_mid;  // (+ the previous merge's token rewrites in workgroups 1..nba)
    if (c->place_pending && !c->place_mid) flush_place(c);
    c->place_pending = false;
    LAUNCH_T(c, "mid_sel", k_mid_sel, dim3(carry ? 1 + c->nba : 1), dim3(ABLOCK), 0, c->D, par, c->run_end, 0);
  }
  {
    const int G = c->nba - MID_APP;  // (+ the previous merge's posting entries in MID_APP more workgroups)
    LAUNCH_T(c, "mid_find", k_mid_find<false>, dim3(c->nba), dim3(ABLOCK), 0, c->D, par, G, 1);
  }
  c->place_pending = true;
  c->place_mid = true;
  c->gen++;
}

// the Sel record of the last mark launch (after a sync)
int read_sel(geobpe_ctx* c, Sel* out) {
  HIPCHK(c, hipMemcpy(out, c->D.sel + (c->gen & 1), sizeof(Sel), hipMemcpyDeviceToHost));
  return 0;
}

// the state and the decision of the last select in one wait: two async copies
// into pinned memory, one stream synchronisation
int sync_state_sel(geobpe_ctx* c, Sel* out) {
  flush_place(c);
  HIPCHK(c, hipMemcpyAsync(c->h_state, c->D.st, sizeof(State), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->h_sel, c->D.sel + (c->gen & 1), sizeof(Sel), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  *out = *c->h_sel;
  return check_device_error(c);
}

// ---------------------------------------------------------------- late-merge path (tail.h)
bool tail_enabled(const geobpe_ctx* c) {
  return c->tail_thresh > 0 && !c->distributed && !c->replay && !c->collapsed;
}

// device bytes tail_alloc takes for R residues (a collapse checks them before it commits)
int64_t tail_bytes(const geobpe_ctx* c, int64_t R) {
  const int64_t kpool = std::min<int64_t>(6 * R + 65536, INT32_MAX - 1) * 4;
  const int64_t tm = (R / 2 + 1024 + MSEG_TM) * (int64_t)sizeof(int4);
  const int64_t thc = R + 2048 + MSEG_TH;
  const int64_t th = thc * (2 * (int64_t)sizeof(int2) + (int64_t)sizeof(int4) + 4 + (int64_t)sizeof(NewPair));
  const int64_t keyed = c->D.kp_off ? 0 : 3 * c->D.HC * 4 + 2 * NBA_MAX * (int64_t)sizeof(int4) + 2 * NBA_MAX * (MID_APP + 1) * 4;
  return kpool + tm + th + keyed;
}

int tail_alloc(geobpe_ctx* c) {
  if (c->tail_ready) return 0;
  Dev& D = c->D;
  D.KPOOL = std::min<int64_t>(6 * c->R + 65536, INT32_MAX - 1);
  D.TMcap = c->R / 2 + 1024 + MSEG_TM;  // (mid.h: the find workgroups' segments, then the spill list)
  D.THcap = c->R + 2048 + MSEG_TH;
  int rc;
  // (zero: a key claimed after the list build starts with an empty list of capacity 0; the
  // key-indexed arrays outlive a collapse, the residue-sized ones are made again for it)
  if (!D.kp_off && ((rc = dalloc(c, &D.kp_off, D.HC, 0)) || (rc = dalloc(c, &D.kp_n, D.HC, 0)) ||
                    (rc = dalloc(c, &D.kp_cap, D.HC, 0)) || (rc = dalloc(c, &D.mcnt, 2 * NBA_MAX, 0)) ||
                    (rc = dalloc(c, &D.mbk, 2 * NBA_MAX * (MID_APP + 1), 0))))
    return rc;
  if ((rc = dalloc(c, &D.kpool, D.KPOOL, 0xFF)) || (rc = dalloc(c, &D.TM, D.TMcap)) || (rc = dalloc(c, &D.TH, 2 * D.THcap)) ||
      (rc = dalloc(c, &D.TS, D.THcap)) || (rc = dalloc(c, &D.TR, D.THcap)) || (rc = dalloc(c, &D.TK, D.THcap)))
    return rc;
  c->tail_ready = true;
  return 0;
}

// per-key posting lists of the live pairs, after any pending place: a counting build with a
// global atomic per key and round of a block (k_kp_alloc / k_kp_fill).  (Round 4 A/B: a stable radix sort of the
// (key, slot) pairs -> runs -> list space -> placement took as long, and its first call loaded
// the sort's code object inside the loop: 25.3k vs 28.6k merges/s end to end)
void tail_build(geobpe_ctx* c) {
  flush_place(c);
  Timed t(c, "tail_build");
  if (c->distributed) {  // (a rank's counts are global: count its own live pairs)
    hipLaunchKernelGGL(k_kp_reset, dim3(c->nb), dim3(BLOCK), 0, c->stream, c->D);
    hipLaunchKernelGGL(k_kp_count, dim3(c->nb), dim3(BLOCK), 0, c->stream, c->D);
  } else {
    hipMemsetAsync(&c->D.st->kpool_used, 0, 8, c->stream);
  }
  hipLaunchKernelGGL(k_kp_alloc, dim3(c->nb), dim3(BLOCK), 0, c->stream, c->D, c->distributed ? 0 : 1);
  hipLaunchKernelGGL(k_kp_fill, dim3(3 * c->nba), dim3(KPF_T), 0, c->stream, c->D);
  hipLaunchKernelGGL(k_mid_flushed, dim3(1), dim3(64), 0, c->stream, c->D);  // (nothing pending)
}

// up to n merges in k_tail (one workgroup, one launch for many merges); a hot-list rebuild
// or the end is run by k_commit on the parity the tail stopped at; stale lists are rebuilt
int tail_run(geobpe_ctx* c, int64_t n) {
  c->enq++;
  int rc;
  if ((rc = tail_alloc(c)) || (rc = sync_state(c))) return rc;
  const int32_t it0 = c->h_state->iter;
  while (!c->h_state->done) {
    const int64_t left = n - (c->h_state->iter - it0);
    if (left <= 0) break;
    if (!c->h_state->kp_valid) tail_build(c);
    const int32_t before = c->h_state->iter;
    {
      Timed t(c, "tail");
      hipLaunchKernelGGL(k_tail, dim3(1), dim3(SBLOCK), 0, c->stream, c->D, (int)(c->gen & 1), left);
    }
    HIPCHK(c, hipGetLastError());
    if ((rc = sync_state(c))) return rc;
    c->gen += c->h_state->iter - before;  // (one launch parity per merge)
    if (c->h_state->tail_exit > 0) {  // an iteration that is no merge: rebuild / measure / done
      Timed t(c, "commit");
      hipLaunchKernelGGL(k_commit<false>, dim3(c->nba), dim3(ABLOCK), 0, c->stream, c->D, 0, (int)(c->gen & 1));
      c->gen++;
      HIPCHK(c, hipGetLastError());
      if ((rc = sync_state(c))) return rc;
    }
  }
  return 0;
}

// (multi-rank: inside the pipelined exchange only -- its iterations write delta records)
bool mid_enabled(const geobpe_ctx* c) {
  return c->mid_thresh > 0 && !c->replay && (!c->distributed || c->pipelined) && c->nba > MID_APP;
}

// a collapsed engine (x_collapse) holds the whole corpus in the token records, the junction
// symbols and the row offsets only: every other residue-sized buffer (rsym, pk, posting index,
// find regions, ...) and the capacities derived from them keep the shard's size, so the
// full-grid kernels (k_select / k_find / k_commit / k_place, the bin pass) must never run on
// it -- only the middle regime, whose arrays are made again for the whole corpus
bool collapsed_grid(const geobpe_ctx* c) { return c->collapsed && !(c->mid_on && mid_enabled(c)); }

// the next batch of iterations before the regime switches are checked (the check is a host
// round trip, ~33 us).  A merge's count falls roughly geometrically, so the merges left before
// the switch are predicted from the last pulled batch's decay, and the batch runs to that
// prediction + 8: overshooting the middle-regime threshold by a few merges costs nothing
// measurable (the regimes run equally fast between 32 768 and 65 536 occurrences),
// while round 4's 8-merge batches near it put three round trips into the driver's window
int64_t tail_batch(const geobpe_ctx* c, int64_t want) {
  const bool mid = mid_enabled(c) && !c->mid_on, tail = tail_enabled(c);
  if (!mid && !tail) return want;
  const int64_t th = mid ? c->mid_thresh : c->tail_thresh;
  const int64_t m = c->h_state->maxc;
  if (m == 0) return std::min<int64_t>(want, 16);
  if (m > 8 * th) return std::min<int64_t>(want, 64);
  // (2 th -> th takes ~20 merges on C3, each 0.964 of the last: 32 overshoots by ~12 merges into
  // the range where the two regimes run equally fast)
  int64_t b = m > 4 * th ? 48 : (m > 2 * th ? 32 : (4 * m > 5 * th ? 16 : 8));
  if (c->decay > 0 && c->decay < 1 && m > th) {
    const double k = std::log((double)th / (double)m) / std::log(c->decay);
    b = std::max<int64_t>(b, std::min<int64_t>(64, (int64_t)k + 8));
  }
  return std::min(want, b);
}
void tail_check_switch(geobpe_ctx* c) {
  const int64_t m = c->h_state->maxc;
  if (m <= 0) return;
  if (mid_enabled(c) && m <= c->mid_thresh) c->mid_on = true;
  if (tail_enabled(c) && m <= c->tail_thresh) c->tail_on = true;
}

// the middle / late regimes' arrays (per-key lists, pool, merged-occurrence and new-pair
// lists: ~90 B per residue) reserved with the key arrays, after the bin pass, so that the
// switch itself allocates nothing (hipMalloc + fill of ~1 GB at C3, inside the merge loop
// otherwise).  A sharded run reserves its shard's here too (round 5 allocated them at the switch,
// inside the sharded loop: ~1 ms at half of C3, in the N = 2 driver window) and again at its
// collapse, for the gathered corpus.
int regime_reserve(geobpe_ctx* c) {
  if (c->mid_thresh <= 0 && c->tail_thresh <= 0) return 0;
  int rc;
  if ((rc = tail_alloc(c))) return rc;
  return sync_state(c);
}

// per-key lists usable by the middle regime: built at the switch, rebuilt when a place
// lost entries (the stalled iterations merged nothing) or the pool is 3/4 used
int mid_prepare(geobpe_ctx* c) {
  int rc;
  if ((rc = tail_alloc(c))) return rc;
  if (!c->h_state->kp_valid || c->h_state->kpool_used > c->D.KPOOL / 4 * 3) tail_build(c);
  return 0;
}

// back to the full-grid kernels (the host-stepped multi-rank path): everything pending is
// placed, the full-grid posting index and the per-key lists are marked stale (each is
// rebuilt when its path runs again)
int mid_leave(geobpe_ctx* c) {
  if (!c->mid_on) return 0;
  flush_place(c);
  HIPCHK(c, hipMemsetAsync(&c->D.st->post_valid, 0, 4, c->stream));
  HIPCHK(c, hipMemsetAsync(&c->D.st->kp_valid, 0, 4, c->stream));
  // k_commit zeroes only the other parity's overflow counters: the last full-grid merge
  // before the switch left its own, which the next find of that parity would extend
  HIPCHK(c, hipMemsetAsync(c->D.st->L_ovf2, 0, sizeof c->D.st->L_ovf2, c->stream));
  HIPCHK(c, hipMemsetAsync(c->D.st->nko2, 0, sizeof c->D.st->nko2, c->stream));
  c->mid_on = false;
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
  HIPCHK(c, hipHostMalloc((void**)&c->h_sel, sizeof(Sel), hipHostMallocDefault));
  memset(c->h_state, 0, sizeof(State));
  c->h_state->place_par = -1;
  int rc;
  if ((rc = dalloc(c, &c->D.st, 1, 0)) || (rc = dalloc(c, &c->D.sel, 2, 0))) return rc;
  HIPCHK(c, hipMemcpyAsync(c->D.st, c->h_state, sizeof(State), hipMemcpyHostToDevice, c->stream));
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    c->ncu = prop.multiProcessorCount;
  c->nba = std::min(c->ncu, NBA_MAX);
  if (const char* e = getenv("GEOBPE_NBA")) {  // (A/B: merge workgroups other than one per CU)
    const int v = atoi(e);
    if (v >= 8 && v <= NBA_MAX) c->nba = v;
  }
  if (const char* e = getenv("GEOBPE_TAIL")) c->tail_thresh = atoll(e);  // (A/B: 0 = never)
  if (const char* e = getenv("GEOBPE_MID")) c->mid_thresh = atoll(e);    // (A/B: 0 = never)
  if (const char* e = getenv("GEOBPE_COLLAPSE_AT")) c->x_collapse_at = atoll(e);  // (A/B: the collapse count)
  if (const char* e = getenv("GEOBPE_XSHARDS")) c->x_shards = std::max<int64_t>(1, atoll(e));  // (bench --shard-of N)
  if (const char* e = getenv("GEOBPE_SPEC")) c->spec = std::max(0, atoi(e));  // (A/B: 0 = no idle iterations)
  c->nb = 8 * c->nba;
  c->D.NB = c->nb;
  c->D.NBA = c->nba;
  return 0;
}

void geobpe_destroy(geobpe_ctx* c) {
  if (!c) return;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  for (void* p : c->allocs) hipFree(p);
  if (c->ev) hipFree(c->ev);
  if (c->ev_n) hipFree(c->ev_n);
  if (c->replay) hipFree(c->replay);
  for (int i = 0; i < 9; i++)
    if (c->d_cols[i]) hipFree(c->d_cols[i]);
  if (c->h_state) hipHostFree(c->h_state);
  if (c->h_sel) hipHostFree(c->h_sel);
  if (c->h_log) hipHostFree(c->h_log);
  for (int q = 0; q < XPEER_MAX; q++)  // (the peers' areas, mapped here by IPC handle)
    if (c->x_peers[q] && c->x_peers[q] != c->x_recv) hipIpcCloseMemHandle(c->x_peers[q]);
  if (c->x_recv) hipFree(c->x_recv);
  if (c->comm && c->rccl.CommDestroy) c->rccl.CommDestroy(c->comm);
  for (uint8_t* p : {c->x_pbuf, c->x_gath, c->x_tmp, c->x_flat})
    if (p) hipFree(p);
  if (c->x_hsend) hipHostFree(c->x_hsend);
  if (c->x_hlog) hipHostFree(c->x_hlog);
  if (c->x_hbeg) hipHostFree(c->x_hbeg);
  if (c->x_hrecv) hipHostFree(c->x_hrecv);
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
  if (c->Lmax >= 65535) return fail(c, GEOBPE_EARG, "chain of %lld residues (token lengths are 16-bit)", (long long)c->Lmax);
  c->R = c->row_off[n_rows];
  if (c->R >= INT32_MAX / 4) return fail(c, GEOBPE_EARG, "too many residues for int32 indexing");
  Dev& D = c->D;
  D.R = c->R;
  D.nrows = n_rows;
  int rc;
  const int64_t Rp = c->R + 8;  // int4 padding for the pk scan
  if ((rc = dalloc(c, &c->d_row_off, n_rows + 1)) || (rc = dalloc(c, &D.rsym, Rp, 0)) ||
      (rc = dalloc(c, &D.gsym, Rp, 0)) || (rc = dalloc(c, &D.tok, Rp, 0xFF)) || (rc = dalloc(c, &D.lab0, Rp, 0xFF)) ||
      (rc = dalloc(c, &D.pk, Rp, 0xFF)))
    return rc;
  D.row_off = c->d_row_off;
  HIPCHK(c, hipMemcpyAsync(c->d_row_off, h_row_off, (n_rows + 1) * 8, hipMemcpyHostToDevice, c->stream));
  // per-workgroup regions: find region r = residue slots [r*PR, (r+1)*PR) (its
  // merges: <= PR/2 + slack, the rest to the overflow list; their new keys' slots
  // T: 2 per merge); commit / bin / import regions: new pairs, claimed keys, found
  // keys (RC)
  D.PR = (c->R + c->nba - 1) / c->nba;
  D.LC = D.PR / 2 + 4096;
  D.TC = 2 * D.LC;
  D.RC = 2 * D.LC + (int64_t)c->nba * SK + 256;
  D.Lovf_cap = c->R / 2 + 1024;
  D.ovf_cap = c->R + 1024;
  if ((rc = dalloc(c, &D.L, (int64_t)c->nba * D.LC)) || (rc = dalloc(c, &D.Lcnt, c->nba, 0)) ||
      (rc = dalloc(c, &D.Lovf, D.Lovf_cap)) || (rc = dalloc(c, &D.np, (int64_t)c->nba * D.RC)) ||
      (rc = dalloc(c, &D.npcnt, c->nba, 0)) || (rc = dalloc(c, &D.npovf, D.ovf_cap)) ||
      (rc = dalloc(c, &D.ns, (int64_t)c->nba * D.RC)) ||
      (rc = dalloc(c, &D.chk, (int64_t)c->nba * D.RC)) || (rc = dalloc(c, &D.chkcnt, c->nba, 0)))
    return rc;
  // posting index: one residue region per find workgroup; per-owner logs of the
  // pairs made since the last rebuild, in CHUNK-entry chunks of one pool of
  // R + slack entries (a merge makes <= R new pairs; k_select has the index
  // rebuilt before a merge that might not fit)
  {
    int64_t ch = 64;
    while (ch < 4096 && ch * c->nba * 2 < c->R) ch <<= 1;
    D.CHUNK = (int32_t)ch;
  }
  D.POOL_CH = (c->R + D.CHUNK - 1) / D.CHUNK + 2 * (int64_t)c->nba + 1;
  D.MAXCH = (int32_t)D.POOL_CH;
  D.KO_cap = std::max<int64_t>(1 << 16, std::min<int64_t>(c->R, 1 << 20));
  if ((rc = dalloc(c, &D.post, (int64_t)c->nba * D.PR)) || (rc = dalloc(c, &D.poff, (int64_t)c->nba * (NBKT + 1), 0)) ||
      (rc = dalloc(c, &D.pool, D.POOL_CH * D.CHUNK)) || (rc = dalloc(c, &D.pch, (int64_t)c->nba * D.MAXCH)) ||
      (rc = dalloc(c, &D.pnch, c->nba, 0)) || (rc = dalloc(c, &D.pfill, c->nba, 0)) ||
      (rc = dalloc(c, &D.KS, (int64_t)c->nba * c->nba * SK + D.KO_cap)) || (rc = dalloc(c, &D.cntK, 2 * (int64_t)c->nba * c->nba, 0)) ||
      (rc = dalloc(c, &D.DS, (int64_t)c->nba * c->nba * SD)) || (rc = dalloc(c, &D.cntD, (int64_t)c->nba * c->nba, 0)) ||
      (rc = dalloc(c, &D.T, (int64_t)c->nba * D.TC)) || (rc = dalloc(c, &D.Tcnt, c->nba, 0)))
    return rc;
  D.KO = D.KS + (int64_t)c->nba * c->nba * SK;  // (one allocation: a record index into KS covers both)
  const int need[6] = {GEOBPE_COL_PHI, GEOBPE_COL_PSI, GEOBPE_COL_OMEGA, GEOBPE_COL_TAU, GEOBPE_COL_CAC1N,
                       GEOBPE_COL_C1NCA};
  for (int q = 0; q < 6; q++) {
    const int k = need[q];
    if (!h_cols[k]) return fail(c, GEOBPE_EARG, "missing angle column %d", k);
    HIPCHK(c, hipMalloc(&c->d_cols[k], c->R * 8 + 8));
    HIPCHK(c, hipMemcpyAsync(c->d_cols[k], h_cols[k], c->R * 8, hipMemcpyHostToDevice, c->stream));
  }
  // content-hash powers
  const int64_t pwn = 2 * c->Lmax + 8;
  std::vector<u64> p1(pwn), p2(pwn);
  p1[0] = p2[0] = 1;
  for (int64_t i = 1; i < pwn; i++) {
    p1[i] = mulmod61(p1[i - 1], HP1);
    p2[i] = mulmod61(p2[i - 1], HP2);
  }
  u64 *dp1, *dp2;
  if ((rc = dalloc(c, &dp1, pwn)) || (rc = dalloc(c, &dp2, pwn))) return rc;
  HIPCHK(c, hipMemcpyAsync(dp1, p1.data(), pwn * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(dp2, p2.data(), pwn * 8, hipMemcpyHostToDevice, c->stream));
  D.pw1 = dp1;
  D.pw2 = dp2;
  D.pwn = pwn;
  // vocab
  D.KC = c->max_vocab;
  D.VSC = std::max<int64_t>(1 << 24, 4 * D.KC);
  if ((rc = dalloc(c, &D.vh1, D.KC)) || (rc = dalloc(c, &D.vh2, D.KC)) || (rc = dalloc(c, &D.vlen, D.KC)) ||
      (rc = dalloc(c, &D.voff, D.KC + 1, 0)) || (rc = dalloc(c, &D.vsym, D.VSC)) || (rc = dalloc(c, &D.log, D.KC)))
    return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));  // the host buffers above are pageable
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
  if (!D.gs16 && (int64_t)B * B * B + B < 65535) {
    int rc;
    if ((rc = dalloc(c, &D.gs16, c->R + 8, 0xFF))) return rc;
  }
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
  const int nb = (int)std::min<int64_t>((c->R + BLOCK - 1) / BLOCK, c->nb);
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
  c->vocab.assign(K0, {});
  std::vector<u64> vh(K0);
  std::vector<int32_t> vl(K0, 1), vs(K0);
  std::vector<int64_t> vo(K0 + 1);
  std::vector<int> seen(K0, 0);
  for (int32_t s = 0; s < S; s++) {
    const int32_t v = h_label_of_sym[s];
    if (v < 0) continue;
    if (v >= K0) return fail(c, GEOBPE_EARG, "label %d >= K0", v);
    c->vocab[v] = {s};
    vh[v] = (u64)(s + 1) % M61;
    vs[v] = s;
    seen[v] = 1;
  }
  for (int32_t v = 0; v < K0; v++)
    if (!seen[v]) return fail(c, GEOBPE_EARG, "label %d has no symbol", v);
  for (int32_t v = 0; v <= K0; v++) vo[v] = v;
  c->K0 = K0;
  int32_t* dl;
  HIPCHK(c, hipMalloc(&dl, (size_t)S * 4));
  HIPCHK(c, hipMemcpyAsync(dl, h_label_of_sym, (size_t)S * 4, hipMemcpyHostToDevice, c->stream));
  if (K0) {
    HIPCHK(c, hipMemcpyAsync(c->D.vh1, vh.data(), K0 * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->D.vh2, vh.data(), K0 * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->D.vlen, vl.data(), K0 * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->D.vsym, vs.data(), K0 * 4, hipMemcpyHostToDevice, c->stream));
  }
  HIPCHK(c, hipMemcpyAsync(c->D.voff, vo.data(), (K0 + 1) * 8, hipMemcpyHostToDevice, c->stream));
  c->h_state->K = K0;
  HIPCHK(c, hipMemcpyAsync(&c->D.st->K, &c->h_state->K, 4, hipMemcpyHostToDevice, c->stream));
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

int geobpe_set_rank(geobpe_ctx* c, int32_t rank) {
  if (!c || rank < 0 || rank >= PIPE_MAX_WORLD) return GEOBPE_EARG;
  c->rank = rank;
  return 0;
}

int geobpe_set_tail(geobpe_ctx* c, int64_t max_count) {
  if (!c || max_count < 0) return GEOBPE_EARG;
  c->tail_thresh = max_count;
  if (!max_count && c->tail_on) return fail(c, GEOBPE_EARG, "the late-merge path is already in use");
  return 0;
}

int geobpe_set_mid(geobpe_ctx* c, int64_t max_count) {
  if (!c || max_count < 0) return GEOBPE_EARG;
  if (c->collapsed && !max_count) return fail(c, GEOBPE_EARG, "a collapsed engine runs the middle regime only");
  c->mid_thresh = max_count;
  if (!max_count && c->mid_on) return fail(c, GEOBPE_EARG, "the middle-regime path is already in use");
  return 0;
}

int geobpe_set_bin_dense(geobpe_ctx* c, int on) {
  if (!c) return GEOBPE_EARG;
  if (c->keys_ready) return fail(c, GEOBPE_EARG, "set_bin_dense must precede bin()");
  c->bin_dense = on != 0;
  return 0;
}

int geobpe_bin(geobpe_ctx* c) {
  if (!c || !c->K0) return GEOBPE_EARG;
  if (c->keys_ready) return fail(c, GEOBPE_EARG, "bin() twice");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = alloc_keys(c))) return rc;
  const int64_t K0 = c->K0, G = c->D.B3;
  if (c->bin_dense && K0 <= BIN_MAXSYM && G <= BIN_MAXSYM && K0 * G * K0 < (1LL << 31)) {
    // bin_dense.h: sample -> cube shape -> pre-claimed cube keys -> count -> reduce / lists
    const int nbc = c->ncu;  // count / list workgroups (144 KB of LDS each)
    BinWork W{};
    W.K0 = (int32_t)K0;
    W.G = (int32_t)G;
    W.nbc = nbc;
    const int64_t NV = c->R / BIN_VEC;
    W.ool_cap = ((NV + nbc - 1) / nbc) * BIN_VEC + BIN_VEC;
    std::vector<void*> tmp;
    auto tmalloc = [&](auto** p, int64_t n) -> hipError_t {
      void* q = nullptr;
      hipError_t e = hipMalloc(&q, (size_t)std::max<int64_t>(n, 1) * sizeof(**p));
      if (e == hipSuccess) tmp.push_back(q);
      *p = (std::remove_reference_t<decltype(*p)>)q;
      return e;
    };
    hipError_t e = hipSuccess;
    if ((e = tmalloc(&W.hist, K0 + G)) || (e = tmalloc(&W.shape, 2)) || (e = tmalloc(&W.cl_of, K0)) ||
        (e = tmalloc(&W.cg_of, G)) || (e = tmalloc(&W.l_at, K0)) || (e = tmalloc(&W.g_at, G)) ||
        (e = tmalloc(&W.flag, BIN_NC)) || (e = tmalloc(&W.cubemap, BIN_NC)) ||
        (e = tmalloc(&W.partial, (int64_t)nbc * BIN_NC)) || (e = tmalloc(&W.ool, (int64_t)nbc * W.ool_cap)) ||
        (e = tmalloc(&W.ooln, nbc)) || (e = tmalloc(&W.found, (int64_t)nbc * AggOol::N)) ||
        (e = tmalloc(&W.foundn, nbc))) {
      for (void* q : tmp) hipFree(q);
      return fail(c, GEOBPE_EHIP, "bin scratch: %s", hipGetErrorString(e));
    }
    HIPCHK(c, hipMemsetAsync(W.hist, 0, (size_t)(K0 + G) * 4, c->stream));
    HIPCHK(c, hipMemsetAsync(W.flag, 0, (size_t)BIN_NC * 4, c->stream));
    const int64_t DS = K0 * G * K0;
    const bool dense_lists = DS <= (1LL << 26);
    if (dense_lists) {
      W.DS = DS;
      W.newcap = std::min<int64_t>(DS, c->R + 1);
      if ((e = tmalloc(&W.dcnt, DS)) || (e = tmalloc(&W.newl, W.newcap)) || (e = tmalloc(&W.nnew, 1))) {
        for (void* q : tmp) hipFree(q);
        return fail(c, GEOBPE_EHIP, "bin scratch: %s", hipGetErrorString(e));
      }
      HIPCHK(c, hipMemsetAsync(W.dcnt, 0, (size_t)DS * 4, c->stream));
      HIPCHK(c, hipMemsetAsync(W.nnew, 0, 8, c->stream));
    }
    {
      Timed t(c, "bin_sample");
      hipLaunchKernelGGL(k_bin_sample, dim3(nbc), dim3(ABLOCK), 0, c->stream, c->D, W);
      hipLaunchKernelGGL(k_bin_rank, dim3(1), dim3(ABLOCK), 0, c->stream, c->D, W);
      hipLaunchKernelGGL(k_bin_flag, dim3(nbc), dim3(ABLOCK), 0, c->stream, c->D, W);
      hipLaunchKernelGGL(k_bin_precube, dim3(BIN_NC / BLOCK), dim3(BLOCK), 0, c->stream, c->D, W);
    }
    {
      Timed t(c, "pair_count");
      hipLaunchKernelGGL(k_bin_count, dim3(nbc), dim3(ABLOCK), 0, c->stream, c->D, W);
    }
    {
      Timed t(c, "bin_claim");
      hipLaunchKernelGGL(k_bin_reduce, dim3(BIN_NC / ABLOCK, (nbc + BIN_RROWS - 1) / BIN_RROWS), dim3(ABLOCK), 0,
                         c->stream, c->D, W, c->distributed ? 1 : 0);
    }
    {
      Timed t(c, "bin_assign");
      if (dense_lists) {
        hipLaunchKernelGGL(k_bin_ool_stage, dim3(nbc), dim3(ABLOCK), 0, c->stream, c->D, W);
        hipLaunchKernelGGL(k_bin_ool_claim, dim3(4 * c->ncu), dim3(BLOCK), 0, c->stream, c->D, W,
                           c->distributed ? 1 : 0);
        hipLaunchKernelGGL(k_bin_ool_fix, dim3(nbc), dim3(ABLOCK), 0, c->stream, c->D, W);
      } else {
        hipLaunchKernelGGL(k_bin_ool, dim3(nbc), dim3(ABLOCK), 0, c->stream, c->D, W, c->distributed ? 1 : 0);
        hipLaunchKernelGGL(k_bin_verify, dim3(nbc), dim3(ABLOCK), 0, c->stream, c->D, W);
      }
    }
    enqueue_pack(c);
    HIPCHK(c, hipGetLastError());
    rc = sync_state(c);
    if (!rc) {
      int32_t shape[2];
      HIPCHK(c, hipMemcpy(shape, W.shape, sizeof shape, hipMemcpyDeviceToHost));
      c->bin_cube[0] = shape[0];
      c->bin_cube[1] = shape[1];
    }
    for (void* q : tmp) hipFree(q);
    return rc ? rc : regime_reserve(c);
  }
  if ((rc = reset_region_counters(c))) return rc;
  {
    Timed t(c, "pair_count");
    hipLaunchKernelGGL(k_pairs_all, dim3(c->nba), dim3(ABLOCK), 0, c->stream, c->D);
  }
  HIPCHK(c, hipGetLastError());
  enqueue_commit(c, c->distributed);
  enqueue_pack(c);
  HIPCHK(c, hipGetLastError());
  if ((rc = sync_state(c))) return rc;
  return regime_reserve(c);
}

int geobpe_step_select(geobpe_ctx* c, int32_t* new_id, int32_t* count) {
  if (!c || !c->keys_ready || !new_id) return GEOBPE_EARG;
  if (c->collapsed) return fail(c, GEOBPE_EARG, "a collapsed engine runs the middle regime only (geobpe_run)");
  if (c->mark_pending) return fail(c, GEOBPE_EARG, "step_select twice without step_apply");
  if (c->pipelined) return fail(c, GEOBPE_EARG, "step_select inside a pipelined exchange");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = mid_leave(c))) return rc;
  Sel sel;
  for (;;) {
    enqueue_select(c);
    HIPCHK(c, hipGetLastError());
    if ((rc = sync_state_sel(c, &sel))) return rc;
    if (sel.decision == SEL_MERGE) break;
    enqueue_apply(c);  // a rebuild iteration (rank-local: every rank then selects the same winner) or done
    if (sel.decision == SEL_DONE) {
      if ((rc = sync_state(c))) return rc;
      *new_id = -1;
      if (count) *count = 0;
      return 0;
    }
  }
  c->mark_pending = true;
  *new_id = sel.nid;
  if (count) *count = sel.maxc;
  return 0;
}

int geobpe_step_apply(geobpe_ctx* c, int64_t* n_merged) {
  if (!c || !c->keys_ready) return GEOBPE_EARG;
  if (!c->mark_pending) return fail(c, GEOBPE_EARG, "step_apply without step_select");
  HIPCHK(c, hipSetDevice(c->device));
  enqueue_mark(c);
  enqueue_apply(c);
  c->mark_pending = false;
  HIPCHK(c, hipGetLastError());
  if (n_merged) {
    int rc;
    if ((rc = sync_state(c))) return rc;
    LogRec lr;
    HIPCHK(c, hipMemcpy(&lr, c->D.log + (c->h_state->iter - 1), sizeof lr, hipMemcpyDeviceToHost));
    *n_merged = lr.nmerged;
  }
  return 0;
}

int geobpe_step(geobpe_ctx* c, int32_t* new_id, int32_t* count, int64_t* n_merged) {
  if (!c || !new_id) return GEOBPE_EARG;
  if (!c->keys_ready) return fail(c, GEOBPE_EARG, "bin() first");
  if (collapsed_grid(c)) return fail(c, GEOBPE_EARG, "a collapsed engine runs the middle regime only");
  if (c->distributed) return fail(c, GEOBPE_EARG, "geobpe_step in distributed mode: use step_select/apply + deltas");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = sync_state(c))) return rc;
  const int32_t it0 = c->h_state->iter;
  if (c->tail_on && tail_enabled(c)) {
    if ((rc = tail_run(c, 1))) return rc;
  } else {
    for (;;) {  // a rebuild (or stalled) iteration merges nothing: go again
      const bool mid = c->mid_on && mid_enabled(c);
      if (mid) {
        if ((rc = mid_prepare(c))) return rc;
        enqueue_iteration_mid(c);
      } else {
        enqueue_iteration(c);
      }
      HIPCHK(c, hipGetLastError());
      if ((rc = sync_state(c))) return rc;
      if (c->h_state->iter != it0 || c->h_state->done) break;
    }
    tail_check_switch(c);
  }
  if (c->h_state->iter == it0) {
    *new_id = -1;
    if (count) *count = 0;
    if (n_merged) *n_merged = 0;
    return 0;
  }
  LogRec lr;
  HIPCHK(c, hipMemcpy(&lr, c->D.log + it0, sizeof lr, hipMemcpyDeviceToHost));
  *new_id = lr.nid;
  if (count) *count = lr.count;
  if (n_merged) *n_merged = lr.nmerged;
  return 0;
}

// the batch loop of geobpe_run; pull: each batch's merge-log records ride to the pinned
// mirror in the batch's own state synchronisation (no extra round trip for the log)
static int run_batches(geobpe_ctx* c, int64_t n_iters, int64_t* n_done, bool pull) {
  if (!c || n_iters < 0) return GEOBPE_EARG;
  if (!c->keys_ready) return fail(c, GEOBPE_EARG, "bin() first");
  if (c->distributed) return fail(c, GEOBPE_EARG, "geobpe_run in distributed mode");
  if (collapsed_grid(c)) return fail(c, GEOBPE_EARG, "a collapsed engine runs the middle regime only");
  HIPCHK(c, hipSetDevice(c->device));
  const int32_t it0 = c->h_state->iter;
  int rc;
  // hot-list rebuild iterations merge nothing: top up until n merges or done; the small
  // merges go to the one-workgroup path
  for (int64_t want = n_iters; want > 0;) {
    if (c->tail_on && tail_enabled(c)) {
      if ((rc = tail_run(c, want))) return rc;
      break;
    }
    const bool mid = c->mid_on && mid_enabled(c);
    if (mid && (rc = mid_prepare(c))) return rc;
    const int64_t batch = tail_batch(c, want);
    // the run's last batch: spec more iterations, which idle on the device once the batch's
    // merges are made (a hot-list rebuild iteration inside the batch then needs no top-up)
    const int64_t extra = batch == want && !c->replay ? c->spec : 0;
    c->run_end = extra ? (int32_t)(c->h_state->iter + batch + 1) : 0;
    if (c->hold_us > 0) hipLaunchKernelGGL(k_hold, dim3(1), dim3(64), 0, c->stream, (int64_t)(100 * c->hold_us));
    for (int64_t i = 0; i < batch + extra; i++) {
      if (mid)
        enqueue_iteration_mid(c);
      else
        enqueue_iteration(c);
    }
    c->run_end = 0;
    HIPCHK(c, hipGetLastError());
    if (pull) {  // (every record this batch can write: <= one per iteration; after the pending
                 // place, which sums the last merge's merged total into its record)
      flush_place(c);
      const int64_t from = c->h_state->iter, n = std::min<int64_t>(batch, c->h_log_cap - from);
      if (n > 0)
        HIPCHK(c, hipMemcpyAsync(c->h_log + from, c->D.log + from, n * sizeof(LogRec), hipMemcpyDeviceToHost,
                                 c->stream));
    }
    const int32_t before = pull ? (int32_t)std::min<int64_t>(c->h_state->iter, c->h_log_cap) : 0;
    if ((rc = sync_state(c))) return rc;
    if (pull) {  // the count's decay over the batch's merges (the next batch's size)
      const int32_t a = before, z = (int32_t)std::min<int64_t>(c->h_state->iter, c->h_log_cap) - 1;
      if (z > a && c->h_log[a].count > 0 && c->h_log[z].count > 0)
        c->decay = std::pow((double)c->h_log[z].count / (double)c->h_log[a].count, 1.0 / (double)(z - a));
    }
    if (c->h_state->done) break;
    tail_check_switch(c);
    want = n_iters - (c->h_state->iter - it0);
  }
  if (n_done) *n_done = c->h_state->iter - it0;
  return 0;
}

int geobpe_run(geobpe_ctx* c, int64_t n_iters, int64_t* n_done) { return run_batches(c, n_iters, n_done, false); }

int geobpe_run_log(geobpe_ctx* c, int64_t n_iters, int64_t* n_done, int64_t* first, int64_t* h_out, int64_t cap) {
  if (!c || !n_done || !first || (cap > 0 && !h_out)) return GEOBPE_EARG;
  if (!c->keys_ready) return fail(c, GEOBPE_EARG, "bin() first");
  const int64_t it0 = c->h_state->iter;
  // the pinned mirror covers every record this run can write (grown by doubling, at most the
  // log's capacity): a run of K merges from merge it0 needs it0 + K + 1
  const int64_t need = std::min<int64_t>(c->D.KC, it0 + n_iters + 1);
  if (need > c->h_log_cap) {
    const int64_t cap = std::min<int64_t>(c->D.KC, std::max<int64_t>({need, 2 * c->h_log_cap, 4096}));
    LogRec* p = nullptr;
    HIPCHK(c, hipHostMalloc((void**)&p, (size_t)cap * sizeof(LogRec), hipHostMallocDefault));
    if (c->h_log) {
      memcpy(p, c->h_log, (size_t)c->h_log_cap * sizeof(LogRec));
      hipHostFree(c->h_log);
    }
    c->h_log = p;
    c->h_log_cap = cap;
  }
  *first = it0;
  int rc;
  if ((rc = run_batches(c, n_iters, n_done, true))) return rc;
  const int64_t n = std::min(*n_done, cap);
  if (c->tail_on && tail_enabled(c) && n > 0)  // (the one-workgroup path syncs on its own: one copy)
    HIPCHK(c, hipMemcpy(c->h_log + it0, c->D.log + it0, n * sizeof(LogRec), hipMemcpyDeviceToHost));
  for (int64_t i = 0; i < n; i++) {
    const LogRec& r = c->h_log[it0 + i];
    h_out[3 * i] = r.nid;
    h_out[3 * i + 1] = r.count;
    h_out[3 * i + 2] = r.nmerged;
  }
  return 0;
}

int64_t geobpe_merge_log(geobpe_ctx* c, int64_t* h_out, int64_t cap) {
  if (!c || !c->keys_ready) return -1;
  if (sync_state(c)) return -1;
  const int64_t n = c->h_state->iter;
  if (h_out && cap > 0) {
    const int64_t m = std::min(n, cap);
    std::vector<LogRec> lr(m);
    if (m && hipMemcpy(lr.data(), c->D.log, m * sizeof(LogRec), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    for (int64_t i = 0; i < m; i++) {
      h_out[3 * i] = lr[i].nid;
      h_out[3 * i + 1] = lr[i].count;
      h_out[3 * i + 2] = lr[i].nmerged;
    }
  }
  return n;
}

int geobpe_delta_export(geobpe_ctx* c, void* d_out, int64_t cap, int64_t* n_records) {
  if (!c || !c->distributed || !n_records) return GEOBPE_EARG;
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = sync_state(c))) return rc;
  const int64_t n = c->h_state->ntouched;
  *n_records = n;
  if (n > cap)
    return fail(c, GEOBPE_ECAPACITY, "delta export needs %lld records (cap %lld)", (long long)n, (long long)cap);
  if (n > 0) hipLaunchKernelGGL(k_export, dim3(c->nb), dim3(BLOCK), 0, c->stream, c->D, (DeltaRec*)d_out, n);
  HIPCHK(c, hipGetLastError());
  c->h_state->epoch += 1;  // new epoch: every key may be touched again
  HIPCHK(c, hipMemcpyAsync(&c->D.st->epoch, &c->h_state->epoch, 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemsetAsync(&c->D.st->ntouched, 0, 8, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

static int delta_import(geobpe_ctx* c, const void* d_in, int64_t n_records) {
  HIPCHK(c, hipSetDevice(c->device));
  const int64_t chunk = (int64_t)c->nba * (c->D.RC - 256);
  int rc;
  for (int64_t off = 0; off < n_records; off += chunk) {
    const int64_t n = std::min(chunk, n_records - off);
    if ((rc = reset_region_counters(c))) return rc;
    hipLaunchKernelGGL(k_import, dim3(c->nba), dim3(ABLOCK), 0, c->stream, c->D, (const DeltaRec*)d_in + off, n);
    HIPCHK(c, hipGetLastError());
    enqueue_commit(c, false);
  }
  return 0;
}

int geobpe_delta_import(geobpe_ctx* c, const void* d_in, int64_t n_records) {
  if (!c || !c->distributed) return GEOBPE_EARG;
  int rc;
  if ((rc = delta_import(c, d_in, n_records))) return rc;
  return sync_state(c);
}

int geobpe_delta_export_async(geobpe_ctx* c, void* d_out, int64_t cap, void* d_count) {
  if (!c || !c->distributed || !d_out || !d_count) return GEOBPE_EARG;
  HIPCHK(c, hipSetDevice(c->device));
  hipLaunchKernelGGL(k_export_dev, dim3(c->nb), dim3(BLOCK), 0, c->stream, c->D, (DeltaRec*)d_out, cap, 0,
                     (int64_t*)nullptr);
  hipLaunchKernelGGL(k_export_fin, dim3(1), dim3(1), 0, c->stream, c->D, (int64_t*)d_count, cap);
  HIPCHK(c, hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------- pipelined exchange
// N > 1 without host waits: per iteration the select / mark / apply triple (launch
// parity kept on the device, State.dgen), the export into a fixed slot (header +
// records), a collective by the caller, and the import of the gathered slots.
// A slot that overflowed stalls every pipelined kernel until the host resolves
// that merge with a sized exchange; the host polls every few iterations.
}  // extern "C"
namespace {
// the pipeline's start: the device's parity counter from the host's, no stall.  lite: without a
// synchronisation when the host state is current (no iteration enqueued since the last sync) --
// the two writes then go out from a pinned pair, stream-ordered before the first select
int pipeline_begin_impl(geobpe_ctx* c, bool lite) {
  if (!c || !c->distributed || !c->keys_ready) return GEOBPE_EARG;
  if (c->mark_pending) return fail(c, GEOBPE_EARG, "pipeline_begin between step_select and step_apply");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if (lite && !c->x_hbeg) HIPCHK(c, hipHostMalloc((void**)&c->x_hbeg, 2 * sizeof(int32_t), hipHostMallocDefault));
  if (lite && c->enq == c->enq_synced && !c->place_pending) {
    c->x_hbeg[0] = (int32_t)c->gen - 1;
    c->x_hbeg[1] = 0;
    c->h_state->dgen = c->x_hbeg[0];
    c->h_state->stall = 0;
    HIPCHK(c, hipMemcpyAsync(&c->D.st->dgen, &c->x_hbeg[0], 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(&c->D.st->stall, &c->x_hbeg[1], 4, hipMemcpyHostToDevice, c->stream));
    c->pipelined = true;
    return 0;
  }
  if ((rc = sync_state(c))) return rc;
  c->h_state->dgen = (int32_t)c->gen - 1;  // the next device iteration takes parity gen & 1
  c->h_state->stall = 0;
  HIPCHK(c, hipMemcpyAsync(&c->D.st->dgen, &c->h_state->dgen, 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(&c->D.st->stall, &c->h_state->stall, 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->pipelined = true;
  return 0;
}
}  // namespace
extern "C" {

int geobpe_pipeline_begin(geobpe_ctx* c) { return pipeline_begin_impl(c, false); }

}  // extern "C"
namespace {
// geobpe_pipeline_end when the last poll has synchronised everything (nothing enqueued since)
int pipeline_end_lite(geobpe_ctx* c) {
  if (c->h_state->stall) return fail(c, GEOBPE_EARG, "pipeline_end while stalled");
  c->gen = (int64_t)c->h_state->dgen + 1;  // host parity continues the device's
  c->pipelined = false;
  return 0;
}
}  // namespace
extern "C" {

}  // extern "C"
namespace {

// the peer exchange's view of producer launch h (exchange.h): every rank's receive area at
// parity h & 1 as mapped here, the launch's sequence number
Dev x_peer_dev(const geobpe_ctx* c, Dev D, int64_t h) {
  D.xw = c->x_world;
  D.xme = c->x_rank;
  D.xrecv = c->x_recv;
  D.xslot = c->x_slot;
  D.xcapf = c->x_rcapf;
  D.xseq = (int32_t)h;
  D.xpar = (int32_t)(h & 1);
  D.xloop = c->x_loop ? 1 : 0;
  D.xchk = c->x_chk;
  D.xchkcnt = c->x_chkcnt;
  D.xchkcap = c->x_chkcap;
  for (int q = 0; q < c->x_world; q++) D.xpeer[q] = c->x_peers[q] + (h & 1) * c->x_world * c->x_slot;
  return D;
}

// before the import of the last producer launch (the next select launch, or the drain): the
// stream waits until every peer's slot header carries that launch's sequence number -- on the
// command processor (hipStreamWaitValue32), or where the device lacks it a one-wave kernel
// with a bounded spin
__global__ void k_xwait(Dev D, int32_t par, int32_t seq) {
  const int q = threadIdx.x;
  if (q >= D.xw || q == D.xme) return;
  const XHdr* h = x_hdr(D.xrecv + (int64_t)par * D.xw * D.xslot, D.xslot, q);
  const uint64_t t0 = wall_clock64();
  // (relaxed system-scope loads in the loop -- they miss the caches -- and one acquire after it:
  // an acquire per iteration would invalidate this XCD's L2 under everything else running)
  while (__hip_atomic_load(&h->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
    __builtin_amdgcn_s_sleep(2);
    if (wall_clock64() - t0 > (uint64_t)200000000) {  // (~2 s: a peer that never publishes)
      set_error(D, GEOBPE_ESTATE, -83);
      D.st->stall = 1;
      return;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}
int x_wait_prev(geobpe_ctx* c, const Dev& D) {
  if (!c->x_pending || c->x_world < 2) return 0;
  const int64_t par = c->x_prev_seq & 1;
  if (!c->x_cpwait) {
    hipLaunchKernelGGL(k_xwait, dim3(1), dim3(64), 0, c->stream, D, (int32_t)par, (int32_t)c->x_prev_seq);
    HIPCHK(c, hipGetLastError());
    return 0;
  }
  for (int q = 0; q < c->x_world; q++) {
    if (q == c->x_rank) continue;
    void* seqp = c->x_recv + (par * c->x_world + q) * c->x_slot + offsetof(XHdr, seq);
    HIPCHK(c, hipStreamWaitValue32(c->stream, seqp, (uint32_t)c->x_prev_seq, hipStreamWaitValueGte, 0xFFFFFFFFu));
  }
  return 0;
}

// the select launch's import workgroups: the place workgroups that share the chip with the
// select workgroup (one 1024-thread workgroup per CU: the launch's last one waits for a CU)
int x_nimp(const geobpe_ctx* c) { return std::max(1, c->nba - 1); }

// one pipelined iteration (geobpe_pipeline_iter); peer: the engine's peer exchange
int pipeline_iter_impl(geobpe_ctx* c, void* d_buf, int64_t cap_total, bool peer, int32_t run_end = 0) {
  c->enq++;
  Dev D = c->D;  // find and commit write this rank's delta records into the slot buffer
  D.xrec = reinterpret_cast<DeltaRec*>(d_buf) + 1;  // record 0 is the slot header
  D.xcap = cap_total;
  int64_t* head = reinterpret_cast<int64_t*>(d_buf);
  if (head != c->x_head) {  // a buffer new to this engine: its count starts at 0 (then the import resets it)
    HIPCHK(c, hipMemsetAsync(head, 0, 8, c->stream));
    c->x_head = head;
  }
  D.xcnt = head;  // the records are counted in the slot header: final when the iteration's last kernel ends
  int nimp = 0;
  if (peer) {
    const int64_t h = c->x_hseq++;
    int rc;
    if ((rc = x_wait_prev(c, x_peer_dev(c, D, c->x_prev_seq)))) return rc;
    D = x_peer_dev(c, D, h);
    nimp = x_nimp(c);
    c->x_pending = true;  // (this launch's headers: the next select launch or the drain waits for them)
    c->x_prev_seq = h;
  }
  if (c->mid_on && mid_enabled(c)) {  // the middle regime (mid.h), device parity
    if (c->place_pending && !c->place_mid) flush_place(c);
    c->place_pending = false;
    LAUNCH_T(c, "mid_sel", k_mid_sel, dim3(1 + c->nba), dim3(ABLOCK), 0, D, -1, run_end, nimp);
    LAUNCH_T(c, "mid_find", k_mid_find<true>, dim3(c->nba), dim3(ABLOCK), 0, D, -1, c->nba - MID_APP, 1);
    c->place_pending = true;
    c->place_mid = true;
    HIPCHK(c, hipGetLastError());
    return 0;
  }
  if (c->place_pending && c->place_mid) flush_place(c);
  {
    const bool place = c->place_pending;  // (+ the previous merge's k_place)
    const int grid = place || nimp ? 1 + c->nba : 1;
    c->place_pending = false;
    LAUNCH_T(c, "select", k_select, dim3(grid), dim3(SBLOCK), 0, D, -1, run_end, place ? 1 : 0, nimp);
  }
  LAUNCH_T(c, "find", k_find, dim3(c->nba), dim3(ABLOCK), 0, D, 1, -1);
  LAUNCH_T(c, "commit", k_commit<true>, dim3(c->nba), dim3(ABLOCK), 0, D, 1, -1);
  c->place_pending = true;
  if (c->ev)
    hipLaunchKernelGGL(k_events, dim3(c->nba), dim3(BLOCK), 0, c->stream, c->D, -1, c->ev, c->ev_cap, c->ev_n);
  HIPCHK(c, hipGetLastError());
  return 0;
}

// the last producer launch's records imported on their own (the end of a batch: the host then
// sees complete counts at its poll)
int x_drain(geobpe_ctx* c) {
  if (!c->x_peer_ready || !c->x_pending) return 0;
  Dev D = x_peer_dev(c, c->D, c->x_prev_seq);
  D.xrec = reinterpret_cast<DeltaRec*>(c->x_pbuf) + 1;
  D.xcap = c->x_pcap;
  D.xcnt = reinterpret_cast<int64_t*>(c->x_pbuf);
  int rc;
  if ((rc = x_wait_prev(c, D))) return rc;
  {
    Timed t(c, "xdrain");
    hipLaunchKernelGGL(k_xdrain, dim3(c->nba), dim3(ABLOCK), 0, c->stream, D);
  }
  HIPCHK(c, hipGetLastError());
  c->x_pending = false;
  return 0;
}

// every import region's found keys checked (the end of a peer-exchange run, or its collapse)
void x_check_all(geobpe_ctx* c) {
  Dev D = x_peer_dev(c, c->D, c->x_prev_seq);
  hipLaunchKernelGGL(k_xcheck, dim3(c->nba), dim3(ABLOCK), 0, c->stream, D);
}

}  // namespace
extern "C" {

int geobpe_pipeline_iter(geobpe_ctx* c, void* d_buf, int64_t cap_total) {
  if (!c || !c->pipelined || !d_buf) return GEOBPE_EARG;
  return pipeline_iter_impl(c, d_buf, cap_total, false);
}

int geobpe_pipeline_import(geobpe_ctx* c, const void* d_slots, int32_t world, int64_t cap_fixed) {
  if (!c || !c->pipelined || !d_slots || world < 1 || world > PIPE_MAX_WORLD || cap_fixed < 0) return GEOBPE_EARG;
  {
    Timed t(c, "import");
    hipLaunchKernelGGL(k_import_fixed, dim3(c->nba), dim3(ABLOCK), 0, c->stream, c->D, (const uint8_t*)d_slots, world,
                       cap_fixed, c->rank < world ? c->rank : -1, c->x_head);
  }
  HIPCHK(c, hipGetLastError());
  return 0;
}

// {stalled, merges made, done, largest slot count of the last import}: one wait
int geobpe_pipeline_poll(geobpe_ctx* c, int64_t* h_out4) {
  if (!c || !c->pipelined || !h_out4) return GEOBPE_EARG;
  int rc;
  if ((rc = sync_state(c))) return rc;
  h_out4[0] = c->h_state->stall;
  h_out4[1] = c->h_state->iter;
  h_out4[2] = c->h_state->done;
  h_out4[3] = c->h_state->slot_max;
  HIPCHK(c, hipMemsetAsync(&c->D.st->slot_max, 0, 8, c->stream));  // (the next window's largest)
  return 0;
}

// the stalled merge's deltas of every rank (gathered by the caller from the
// slots' full buffers): import them and release the pipeline
int geobpe_pipeline_resolve(geobpe_ctx* c, const void* d_in, int64_t n_records) {
  if (!c || !c->pipelined) return GEOBPE_EARG;
  int rc;
  if ((rc = delta_import(c, d_in, n_records))) return rc;
  if (c->x_head) HIPCHK(c, hipMemsetAsync(c->x_head, 0, 8, c->stream));  // (the stalled merge's count, consumed)
  HIPCHK(c, hipMemsetAsync(&c->D.st->xpend, 0, 4, c->stream));            // (peer exchange: nothing pending)
  HIPCHK(c, hipMemsetAsync(&c->D.st->stall, 0, 4, c->stream));
  return sync_state(c);
}

int geobpe_pipeline_end(geobpe_ctx* c) {
  if (!c || !c->pipelined) return GEOBPE_EARG;
  int rc;
  if ((rc = sync_state(c))) return rc;
  if (c->h_state->stall) return fail(c, GEOBPE_EARG, "pipeline_end while stalled");
  c->gen = (int64_t)c->h_state->dgen + 1;  // host parity continues the device's
  c->pipelined = false;
  return 0;
}

int geobpe_delta_import_async(geobpe_ctx* c, const void* d_in, int64_t n_records) {
  if (!c || !c->distributed) return GEOBPE_EARG;
  return delta_import(c, d_in, n_records);
}

int64_t geobpe_token_json(geobpe_ctx* c, int32_t v, char* buf, int64_t cap) {
  if (!c) return -1;
  if (v >= (int32_t)c->vocab.size() && sync_vocab(c)) return -1;
  if (v < 0 || v >= (int32_t)c->vocab.size()) return -1;
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
  if (!c) return -1;
  if (v >= (int32_t)c->vocab.size() && sync_vocab(c)) return -1;
  if (v < 0 || v >= (int32_t)c->vocab.size()) return -1;
  const auto& x = c->vocab[v];
  if (h_out) memcpy(h_out, x.data(), sizeof(int32_t) * std::min<int64_t>(cap, (int64_t)x.size()));
  return (int64_t)x.size();
}

int64_t geobpe_vocab_count(geobpe_ctx* c) {
  if (!c) return -1;
  if (!c->R) return (int64_t)c->vocab.size();
  if (sync_state(c)) return -1;
  return c->h_state->K ? c->h_state->K : (int64_t)c->vocab.size();
}

int64_t geobpe_num_keys(geobpe_ctx* c) {
  if (!c || !c->keys_ready) return 0;
  if (sync_state(c)) return -1;
  hipMemsetAsync(&c->D.st->nkeys, 0, 8, c->stream);
  hipLaunchKernelGGL(k_count_keys, dim3(c->nb), dim3(BLOCK), 0, c->stream, c->D);
  if (sync_state(c)) return -1;
  return c->h_state->nkeys;
}

static int row_token_offsets(geobpe_ctx* c, std::vector<int64_t>& off, int64_t** d_off) {
  flush_place(c);
  int64_t* dn;
  HIPCHK(c, hipMalloc(&dn, (c->nrows + 1) * 8));
  hipLaunchKernelGGL(k_row_ntok, dim3(c->nb), dim3(BLOCK), 0, c->stream, c->D, dn);
  std::vector<int64_t> n(c->nrows);
  HIPCHK(c, hipMemcpyAsync(n.data(), dn, c->nrows * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  off.assign(c->nrows + 1, 0);
  for (int64_t r = 0; r < c->nrows; r++) off[r + 1] = off[r] + n[r];
  HIPCHK(c, hipMemcpyAsync(dn, off.data(), (c->nrows + 1) * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  *d_off = dn;
  return 0;
}

int64_t geobpe_debug_state(geobpe_ctx* c, int64_t* h_out, int64_t cap) {
  if (!c || !h_out || cap < 10) return GEOBPE_EARG;
  if (int rc = sync_state(c)) return rc;
  const State& s = *c->h_state;
  const int64_t v[13] = {s.ncl2[s.cl_act], s.theta, s.ncand, s.maxc, s.nskip, s.cl_valid,
                         s.iter, s.K, s.post_valid, s.pool_used, s.stat_krec, s.stat_drec, s.stat_keys};
  const int64_t n = std::min<int64_t>(cap, 13);
  for (int64_t i = 0; i < n; i++) h_out[i] = v[i];
  return n;
}

// the rows this context reports: all of them, or after a collapse its own rank's window
static void own_rows(const geobpe_ctx* c, int64_t* r0, int64_t* r1) {
  *r0 = c->collapsed ? c->own_row0 : 0;
  *r1 = c->collapsed ? c->own_row1 : c->nrows;
}

int64_t geobpe_num_tokens(geobpe_ctx* c) {
  if (!c || !c->R) return -1;
  std::vector<int64_t> off;
  int64_t* d;
  if (row_token_offsets(c, off, &d)) return -1;
  hipFree(d);
  int64_t r0, r1;
  own_rows(c, &r0, &r1);
  return off[r1] - off[r0];
}

int64_t geobpe_segmentation(geobpe_ctx* c, int32_t* h_start, int32_t* h_id, int64_t* h_row_tok_off) {
  if (!c || !c->R) return -1;
  hipSetDevice(c->device);
  std::vector<int64_t> off;
  int64_t* d_off;
  if (row_token_offsets(c, off, &d_off)) return -1;
  int64_t r0, r1;
  own_rows(c, &r0, &r1);
  const int64_t T = off.back(), t0 = off[r0], Tw = off[r1] - off[r0];
  if (h_row_tok_off)
    for (int64_t r = r0; r <= r1; r++) h_row_tok_off[r - r0] = off[r] - t0;
  if (h_start || h_id) {
    int32_t *ds, *di;
    if (hipMalloc(&ds, T * 4 + 4) != hipSuccess || hipMalloc(&di, T * 4 + 4) != hipSuccess) return -1;
    hipLaunchKernelGGL(k_row_seg, dim3(c->nb), dim3(BLOCK), 0, c->stream, c->D, (const int64_t*)d_off, ds, di);
    if (h_start) hipMemcpyAsync(h_start, ds + t0, Tw * 4, hipMemcpyDeviceToHost, c->stream);
    if (h_id) hipMemcpyAsync(h_id, di + t0, Tw * 4, hipMemcpyDeviceToHost, c->stream);
    hipStreamSynchronize(c->stream);
    hipFree(ds);
    hipFree(di);
  }
  hipFree(d_off);
  return Tw;
}

int64_t geobpe_encode(geobpe_ctx* c, int32_t* h_ids, int64_t* h_row_id_off) {
  if (!c || !c->R) return -1;
  hipSetDevice(c->device);
  if (sync_state(c)) return -1;
  const int32_t K = c->h_state->K;
  std::vector<int64_t> off;
  int64_t* d_off;
  if (row_token_offsets(c, off, &d_off)) return -1;
  std::vector<int64_t> ioff(c->nrows + 1, 0);
  for (int64_t r = 0; r < c->nrows; r++) ioff[r + 1] = ioff[r] + 4 * (off[r + 1] - off[r]) - 3;
  int64_t r0, r1;
  own_rows(c, &r0, &r1);
  const int64_t T = ioff.back(), i0 = ioff[r0], Tw = ioff[r1] - ioff[r0];
  if (h_row_id_off)
    for (int64_t r = r0; r <= r1; r++) h_row_id_off[r - r0] = ioff[r] - i0;
  if (h_ids) {
    int32_t* di;
    if (hipMalloc(&di, T * 4 + 4) != hipSuccess) return -1;
    hipMemcpyAsync(d_off, ioff.data(), (c->nrows + 1) * 8, hipMemcpyHostToDevice, c->stream);
    hipLaunchKernelGGL(k_row_encode, dim3(c->nb), dim3(BLOCK), 0, c->stream, c->D, (const int64_t*)d_off, di, K);
    hipMemcpyAsync(h_ids, di + i0, Tw * 4, hipMemcpyDeviceToHost, c->stream);
    hipStreamSynchronize(c->stream);
    hipFree(di);
  }
  hipFree(d_off);
  return Tw;
}

int64_t geobpe_verify_counts(geobpe_ctx* c) {
  if (!c || !c->keys_ready || c->distributed) return -1;
  hipSetDevice(c->device);
  if (sync_state(c)) return -1;
  hipMemsetAsync(c->D.scratch, 0, c->D.HC * 4, c->stream);
  hipMemsetAsync(&c->D.st->nmismatch, 0, 8, c->stream);
  {
    Timed t(c, "recount");
    hipLaunchKernelGGL(k_recount, dim3(c->nb), dim3(BLOCK), 0, c->stream, c->D);
  }
  hipLaunchKernelGGL(k_compare, dim3(c->nb), dim3(BLOCK), 0, c->stream, c->D);
  if (sync_state(c)) return -1;
  return c->h_state->nmismatch;
}

int geobpe_marker(geobpe_ctx* c, int32_t tag) {
  if (!c) return GEOBPE_EARG;
  HIPCHK(c, hipSetDevice(c->device));
  hipLaunchKernelGGL(k_window_mark, dim3(1), dim3(64), 0, c->stream, tag, c->D.st);
  HIPCHK(c, hipGetLastError());
  return 0;
}

int64_t geobpe_debug_timeline(geobpe_ctx* c, int on, int64_t* h_out, int64_t cap) {
  if (!c) return -1;
  if (hipSetDevice(c->device) != hipSuccess) return -1;
  const int64_t n = (int64_t)c->nb * DBG_SLOTS;
  if (on) {
    if (!c->D.dbg && dalloc(c, &c->D.dbg, n)) return -1;
    hipMemsetAsync(c->D.dbg, 0, n * 8, c->stream);
    return n;
  }
  if (!c->D.dbg) return 0;
  hipStreamSynchronize(c->stream);
  if (h_out && cap > 0) hipMemcpy(h_out, c->D.dbg, std::min(cap, n) * 8, hipMemcpyDeviceToHost);
  c->D.dbg = nullptr;  // (the buffer stays allocated until destroy)
  return n;
}

int geobpe_debug_key_less(geobpe_ctx* c, const int32_t* h_pairs, int32_t n, int32_t* h_out) {
  if (!c || !c->keys_ready || n < 0) return GEOBPE_EARG;
  HIPCHK(c, hipSetDevice(c->device));
  int32_t *dp, *dout;
  HIPCHK(c, hipMalloc(&dp, 8 * (size_t)n + 8));
  HIPCHK(c, hipMalloc(&dout, 4 * (size_t)n + 4));
  HIPCHK(c, hipMemcpyAsync(dp, h_pairs, 8 * (size_t)n, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(k_debug_key_less, dim3((64 * (int64_t)n + 255) / 256 + 1), dim3(256), 0, c->stream, c->D, (const int32_t*)dp,
                     dout, n);
  HIPCHK(c, hipMemcpyAsync(h_out, dout, 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  hipFree(dp);
  hipFree(dout);
  return 0;
}

int64_t geobpe_key_json(geobpe_ctx* c, int32_t d, char* buf, int64_t cap) {
  if (!c || !c->keys_ready || d < 0) return -1;
  if (sync_vocab(c)) return -1;
  if (d >= c->D.HC) return -1;
  int32_t rep[3];
  if (hipMemcpy(rep, c->D.krep + 3 * (int64_t)d, sizeof rep, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  const int32_t K = (int32_t)c->vocab.size();
  if (rep[0] < 0 || rep[0] >= K || rep[2] < 0 || rep[2] >= K) return -1;  // not a key
  std::vector<int32_t> x(c->vocab[rep[0]]);
  x.push_back(rep[1]);
  x.insert(x.end(), c->vocab[rep[2]].begin(), c->vocab[rep[2]].end());
  std::string s;
  geobpe::render_key(x.data(), (int64_t)x.size(), c->B, s);
  if (buf && cap > 0) {
    const int64_t m = std::min<int64_t>((int64_t)s.size(), cap - 1);
    memcpy(buf, s.data(), m);
    buf[m] = 0;
  }
  return (int64_t)s.size();
}

int64_t geobpe_debug_counts(geobpe_ctx* c, int32_t* h_keys, int32_t* h_counts, int64_t cap) {
  if (!c || !c->keys_ready) return -1;
  if (sync_state(c)) return -1;
  const int64_t U = std::min(c->h_state->U, c->D.KCAP);
  const int64_t n = std::min(U, cap);
  if (h_keys && h_counts && n > 0) {
    int32_t *dk, *dc;
    if (hipMalloc(&dk, n * 4) != hipSuccess || hipMalloc(&dc, n * 4) != hipSuccess) return -1;
    hipLaunchKernelGGL(k_gather_counts, dim3(c->nb), dim3(BLOCK), 0, c->stream, c->D, dk, dc, n);
    hipMemcpyAsync(h_keys, dk, n * 4, hipMemcpyDeviceToHost, c->stream);
    hipMemcpyAsync(h_counts, dc, n * 4, hipMemcpyDeviceToHost, c->stream);
    hipStreamSynchronize(c->stream);
    hipFree(dk);
    hipFree(dc);
  }
  return U;
}

int geobpe_debug_key(geobpe_ctx* c, int32_t d, int64_t* out) {
  if (!c || !c->keys_ready || d < 0 || !out) return GEOBPE_EARG;
  int rc;
  if ((rc = sync_state(c))) return rc;
  int32_t rep[3], len, cnt, dense = -2;
  u64 h1;
  HIPCHK(c, hipMemcpy(rep, c->D.krep + 3 * (int64_t)d, sizeof rep, hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(&len, c->D.klen + d, 4, hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(&cnt, c->D.count + d, 4, hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(&h1, c->D.kh1 + d, 8, hipMemcpyDeviceToHost));
  out[0] = rep[0];
  out[1] = rep[1];
  out[2] = rep[2];
  out[3] = len;
  out[4] = cnt;
  out[5] = c->h_state->U;
  out[6] = c->h_state->K;
  out[7] = (int64_t)c->vocab.size();
  out[8] = (int64_t)h1;
  (void)dense;
  return 0;
}

int geobpe_set_profiling(geobpe_ctx* c, int on) {
  if (!c) return GEOBPE_EARG;
  collect_events(c);
  c->prof = on > 0;
  c->prof_stride = on > 1 ? on : 1;
  c->D.stats = c->prof && c->prof_stride == 1 ? 1 : 0;  // (work counters only under full profiling)
  c->prof_seen.clear();
  c->ktime.clear();
  // events made now, not at the first sampled launches (hipEventCreate is host work inside
  // the loop being measured)
  if (c->prof) {
    const size_t have = c->evpool.size();
    std::vector<hipEvent_t> made;
    for (size_t i = have; i < 128; i++) made.push_back(make_event(c));
    c->evpool.insert(c->evpool.end(), made.begin(), made.end());
  }
  return 0;
}

int geobpe_set_hold(geobpe_ctx* c, int64_t us) {
  if (!c || us < 0 || us > 1000000) return GEOBPE_EARG;
  c->hold_us = us;
  return 0;
}

int geobpe_set_work_counters(geobpe_ctx* c, int on) {
  if (!c) return GEOBPE_EARG;
  c->D.stats = on ? 1 : 0;
  return 0;
}

int geobpe_set_profiling_filter(geobpe_ctx* c, const char* names) {
  if (!c) return GEOBPE_EARG;
  c->prof_filter = (names && *names) ? "," + std::string(names) + "," : std::string();
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

int geobpe_replay_load(geobpe_ctx* c, const uint64_t* h_h1, const uint64_t* h_h2, const int32_t* h_len,
                       const int32_t* h_idL, const int32_t* h_g, const int32_t* h_idR, int64_t n) {
  if (!c || n < 0 || (n && (!h_h1 || !h_h2 || !h_len || !h_idL || !h_g || !h_idR))) return GEOBPE_EARG;
  if (!c->keys_ready) return fail(c, GEOBPE_EARG, "bin() first");
  if (c->distributed || c->collapsed) return fail(c, GEOBPE_EARG, "merge replay is single-rank");
  if (c->h_state->iter > 0) return fail(c, GEOBPE_EARG, "merge replay must start before the first merge");
  if (c->K0 + n > c->max_vocab) return fail(c, GEOBPE_ECAPACITY, "K0 + %lld merges exceed max_vocab", (long long)n);
  std::vector<ReplayRec> r((size_t)n);
  for (int64_t t = 0; t < n; t++) {
    const int32_t v = c->K0 + (int32_t)t;
    if (h_idL[t] < 0 || h_idL[t] >= v || h_idR[t] < 0 || h_idR[t] >= v || h_len[t] < 2)
      return fail(c, GEOBPE_EARG, "replay record %lld: split (%d, %d) is not of earlier tokens", (long long)t,
                  h_idL[t], h_idR[t]);
    r[t] = ReplayRec{h_h1[t], h_h2[t], h_len[t], h_idL[t], h_g[t], h_idR[t]};
  }
  HIPCHK(c, hipSetDevice(c->device));
  if (c->replay) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(c->replay);
    c->replay = nullptr;
  }
  HIPCHK(c, hipMalloc(&c->replay, std::max<size_t>(1, (size_t)n) * sizeof(ReplayRec)));
  if (n)
    HIPCHK(c, hipMemcpyAsync(c->replay, r.data(), (size_t)n * sizeof(ReplayRec), hipMemcpyHostToDevice, c->stream));
  c->replay_n = n;
  return 0;
}

// ---- PDB -> internal coordinates (featurize.h)
static thread_local std::string g_pdb_err;

const char* geobpe_pdb_error(void) { return g_pdb_err.c_str(); }

int64_t geobpe_pdb_backbone(const char* path, double* h_xyz, int64_t cap_residues) {
  if (!path) return GEOBPE_EARG;
  std::vector<double> xyz;
  g_pdb_err.clear();
  const int n = pdb_backbone(path, xyz, g_pdb_err);
  if (n < 0) return n == -2 ? -(int64_t)GEOBPE_EVALUE : -(int64_t)GEOBPE_EARG;
  if (h_xyz) {
    if (n > cap_residues) {
      g_pdb_err = "buffer too small";
      return -(int64_t)GEOBPE_ECAPACITY;
    }
    std::memcpy(h_xyz, xyz.data(), xyz.size() * sizeof(double));
  }
  return n;
}

int geobpe_featurize(int device, int64_t n_rows, const int64_t* h_row_off, const double* h_xyz,
                     double* const* h_cols) {
  if (n_rows < 0 || !h_row_off || !h_cols) return GEOBPE_EARG;
  const int64_t R = h_row_off[n_rows];
  if (R == 0) return 0;
  if (!h_xyz) return GEOBPE_EARG;
  if (hipSetDevice(device) != hipSuccess) return GEOBPE_EHIP;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return GEOBPE_EHIP;
  int64_t* d_off = nullptr;
  double *d_xyz = nullptr, *d_out = nullptr;
  int rc = 0;
  if (hipMalloc(&d_off, (n_rows + 1) * 8) != hipSuccess || hipMalloc(&d_xyz, R * 9 * 8) != hipSuccess ||
      hipMalloc(&d_out, R * 9 * 8) != hipSuccess) {
    rc = GEOBPE_EHIP;
  } else {
    hipMemcpyAsync(d_off, h_row_off, (n_rows + 1) * 8, hipMemcpyHostToDevice, s);
    hipMemcpyAsync(d_xyz, h_xyz, R * 9 * 8, hipMemcpyHostToDevice, s);
    const int nb = (int)std::min<int64_t>(std::max<int64_t>(n_rows, 1), 65536);
    hipLaunchKernelGGL(k_featurize, dim3(nb), dim3(BLOCK), 0, s, n_rows, (const int64_t*)d_off,
                       (const double*)d_xyz, d_out, R);
    if (hipGetLastError() != hipSuccess) rc = GEOBPE_EHIP;
    for (int col = 0; col < 9 && !rc; col++)
      if (hipMemcpyAsync(h_cols[col], d_out + col * R, R * 8, hipMemcpyDeviceToHost, s) != hipSuccess) rc = GEOBPE_EHIP;
    if (hipStreamSynchronize(s) != hipSuccess) rc = GEOBPE_EHIP;
  }
  hipFree(d_off);
  hipFree(d_xyz);
  hipFree(d_out);
  hipStreamDestroy(s);
  return rc;
}

namespace {
// The context-free entry points (glue opt, NeRF, Kabsch) keep one stream and one scratch arena
// per (device, entry point) for the process, grown on demand: the RMSD mode calls them once or
// twice per key and induce once per chain, where a stream and a few allocations per call used
// to outweigh the kernels.  Each arena has its own lock (calls on different devices or entry
// points run concurrently; calls on one arena are serialised); geobpe_arena_release returns
// the memory and the streams.
struct Arena {
  std::mutex mu;
  hipStream_t s = nullptr;
  char* buf = nullptr;
  size_t cap = 0;
};
std::mutex g_arena_mu;  // guards the map only
std::map<std::pair<int, int>, std::unique_ptr<Arena>> g_arena;
enum { ARENA_GLUE = 0, ARENA_NERF = 1, ARENA_RMSD = 2 };

Arena* arena_of(int device, int which) {
  std::lock_guard<std::mutex> lock(g_arena_mu);
  std::unique_ptr<Arena>& p = g_arena[std::make_pair(device, which)];
  if (!p) p.reset(new Arena());
  return p.get();  // (entries are never erased: the pointer stays valid)
}

// the arena's stream and n buffers of sizes[i] bytes (256-B aligned) in ptr[i]; the caller holds ar.mu
int arena_take(Arena& ar, int n, const size_t* sizes, void** ptr, hipStream_t* s) {
  if (!ar.s && hipStreamCreateWithFlags(&ar.s, hipStreamNonBlocking) != hipSuccess) {
    ar.s = nullptr;
    return GEOBPE_EHIP;
  }
  size_t total = 0;
  for (int i = 0; i < n; i++) total += (sizes[i] + 255) / 256 * 256;
  if (ar.cap < total) {
    if (ar.buf) hipFree(ar.buf);
    ar.buf = nullptr;
    ar.cap = 0;
    const size_t want = total + total / 4;
    if (hipMalloc(&ar.buf, want) != hipSuccess) return GEOBPE_EHIP;
    ar.cap = want;
  }
  char* q = ar.buf;
  for (int i = 0; i < n; i++) {
    ptr[i] = q;
    q += (sizes[i] + 255) / 256 * 256;
  }
  *s = ar.s;
  return 0;
}
}  // namespace

int geobpe_arena_release(int device) {
  std::vector<Arena*> arenas;
  {
    std::lock_guard<std::mutex> lock(g_arena_mu);
    for (auto& kv : g_arena)
      if (device < 0 || kv.first.first == device) arenas.push_back(kv.second.get());
  }
  int rc = 0;
  for (Arena* ar : arenas) {
    std::lock_guard<std::mutex> lock(ar->mu);
    if (ar->s && hipStreamSynchronize(ar->s) != hipSuccess) rc = GEOBPE_EHIP;
    if (ar->buf) hipFree(ar->buf);
    if (ar->s) hipStreamDestroy(ar->s);
    ar->buf = nullptr;
    ar->cap = 0;
    ar->s = nullptr;
  }
  return rc;
}

int geobpe_rmsd(int device, int32_t n_a, int32_t n_b, int32_t n_atoms, const double* h_a, const double* h_b,
                int symmetric, double* h_out) {
  if (n_a < 0 || n_atoms <= 0 || !h_a || !h_out) return GEOBPE_EARG;
  if (symmetric) {
    h_b = h_a;
    n_b = n_a;
  }
  if (n_b < 0 || !h_b) return GEOBPE_EARG;
  if ((int64_t)n_a * n_b == 0) return 0;
  if (hipSetDevice(device) != hipSuccess) return GEOBPE_EHIP;
  const int64_t la = (int64_t)n_a * n_atoms * 3, lb = (int64_t)n_b * n_atoms * 3, no = (int64_t)n_a * n_b;
  double *d_a = nullptr, *d_b = nullptr, *d_out = nullptr;
  Arena& ar = *arena_of(device, ARENA_RMSD);
  std::lock_guard<std::mutex> lock(ar.mu);
  hipStream_t s;
  const size_t sizes[3] = {(size_t)la * 8, symmetric ? 0 : (size_t)lb * 8, (size_t)no * 8};
  void* ptr[3];
  int rc = arena_take(ar, 3, sizes, ptr, &s);
  if (!rc) {
    d_a = (double*)ptr[0];
    d_b = symmetric ? nullptr : (double*)ptr[1];
    d_out = (double*)ptr[2];
    hipMemcpyAsync(d_a, h_a, la * 8, hipMemcpyHostToDevice, s);
    hipLaunchKernelGGL(k_rmsd_center, dim3((n_a + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, d_a, n_a, n_atoms);
    if (!symmetric) {
      hipMemcpyAsync(d_b, h_b, lb * 8, hipMemcpyHostToDevice, s);
      hipLaunchKernelGGL(k_rmsd_center, dim3((n_b + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, d_b, n_b, n_atoms);
    }
    hipLaunchKernelGGL(k_rmsd_pairs, dim3((unsigned)((no + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, (const double*)d_a,
                       (const double*)(symmetric ? d_a : d_b), n_a, n_b, n_atoms, symmetric, d_out);
    if (hipGetLastError() != hipSuccess) rc = GEOBPE_EHIP;
    if (!rc && hipMemcpyAsync(h_out, d_out, no * 8, hipMemcpyDeviceToHost, s) != hipSuccess) rc = GEOBPE_EHIP;
    if (hipStreamSynchronize(s) != hipSuccess) rc = GEOBPE_EHIP;
  }
  return rc;
}

int geobpe_nerf(int device, int64_t n_spans, const int64_t* h_res_off, const double* h_geo, double* h_xyz) {
  if (n_spans < 0 || !h_res_off) return GEOBPE_EARG;
  const int64_t R = h_res_off[n_spans];
  if (R == 0) return 0;
  if (!h_geo || !h_xyz) return GEOBPE_EARG;
  if (hipSetDevice(device) != hipSuccess) return GEOBPE_EHIP;
  int64_t* d_off = nullptr;
  double *d_geo = nullptr, *d_out = nullptr;
  Arena& ar = *arena_of(device, ARENA_NERF);
  std::lock_guard<std::mutex> lock(ar.mu);
  hipStream_t s;
  const size_t sizes[3] = {(size_t)(n_spans + 1) * 8, (size_t)R * 9 * 8, (size_t)R * 9 * 8};
  void* ptr[3];
  int rc = arena_take(ar, 3, sizes, ptr, &s);
  if (!rc) {
    d_off = (int64_t*)ptr[0];
    d_geo = (double*)ptr[1];
    d_out = (double*)ptr[2];
    hipMemcpyAsync(d_off, h_res_off, (n_spans + 1) * 8, hipMemcpyHostToDevice, s);
    hipMemcpyAsync(d_geo, h_geo, R * 9 * 8, hipMemcpyHostToDevice, s);
    hipLaunchKernelGGL(k_nerf, dim3((unsigned)((n_spans + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, n_spans,
                       (const int64_t*)d_off, (const double*)d_geo, d_out);
    if (hipGetLastError() != hipSuccess) rc = GEOBPE_EHIP;
    if (!rc && hipMemcpyAsync(h_xyz, d_out, R * 9 * 8, hipMemcpyDeviceToHost, s) != hipSuccess) rc = GEOBPE_EHIP;
    if (hipStreamSynchronize(s) != hipSuccess) rc = GEOBPE_EHIP;
  }
  return rc;
}

int geobpe_glue_opt(int device, int64_t n_chains, const int64_t* h_res_off, const double* h_geo, const float* h_x0,
                    const float* h_tgt, const int32_t* h_grid, int32_t n_grid, int32_t kmax, const float* h_prior,
                    const int32_t* h_kcnt, float lam, double w_rot, double w_trans, float* h_xout, int32_t* h_stats,
                    double* h_loss) {
  if (n_chains < 0 || !h_res_off) return GEOBPE_EARG;
  if (n_chains == 0) return 0;
  const int64_t R = h_res_off[n_chains];
  int64_t rmax = 0;
  for (int64_t i = 0; i < n_chains; i++) {
    const int64_t r = h_res_off[i + 1] - h_res_off[i];
    if (r < 1) return GEOBPE_EARG;  // (the glue offsets g0 = a0 - s assume >= 1 residue per chain)
    rmax = std::max(rmax, r);
  }
  const int64_t G = R - n_chains;  // glues: r - 1 per chain
  if (R == 0 || G <= 0) return 0;
  if (!h_geo || !h_x0 || !h_tgt || !h_grid || !h_prior || !h_kcnt || !h_xout || !h_stats || !h_loss) return GEOBPE_EARG;
  if (n_grid <= 0 || kmax <= 0) return GEOBPE_EARG;
  for (int64_t i = 0; i < n_chains; i++)
    if (h_grid[i] < 0 || h_grid[i] >= n_grid) return GEOBPE_EARG;
  for (int64_t i = 0; i < 3 * (int64_t)n_grid; i++)
    if (h_kcnt[i] <= 0 || h_kcnt[i] > kmax) return GEOBPE_EARG;
  if (hipSetDevice(device) != hipSuccess) return GEOBPE_EHIP;
  Arena& ar = *arena_of(device, ARENA_GLUE);
  std::lock_guard<std::mutex> lock(ar.mu);  // (the per-device arena: see arena_take)
  hipStream_t s = nullptr;
  const int64_t pmax = 3 * (rmax - 1), S = n_chains;
  GlueProb P{};
  P.S = S;
  P.kmax = kmax;
  P.lam = lam;
  P.wR = w_rot;
  P.wt = w_trans;
  P.pmax = pmax;
  int64_t *d_off = nullptr;
  double *d_geo = nullptr, *d_loss = nullptr;
  float *d_x0 = nullptr, *d_tgt = nullptr, *d_prior = nullptr, *d_xout = nullptr;
  int32_t *d_grid = nullptr, *d_kcnt = nullptr, *d_stats = nullptr;
  int rc = 0;
  // one wave per chain (k_glue_wave, scratch at each chain's residue / glue offset); the
  // one-thread-per-chain k_glue_opt (scratch interleaved over the chains, n_chains x the
  // longest chain) stays as an A/B switch: GEOBPE_GLUE_THREAD=1
  const char* ge = getenv("GEOBPE_GLUE_THREAD");
  const bool wave = !(ge && atoi(ge) == 1);
  const int64_t NG = 3 * G;
  const int64_t nx = wave ? 9 * R : 9 * rmax * S;
  const int64_t nv = wave ? NG : pmax * S;
  const size_t sizes[14] = {(size_t)(S + 1) * 8, (size_t)R * 9 * 8, (size_t)G * 3 * 4, (size_t)G * 12 * 4,
                            (size_t)S * 4, (size_t)n_grid * 6 * kmax * 4, (size_t)n_grid * 3 * 4, (size_t)G * 3 * 4,
                            (size_t)S * 2 * 4, (size_t)S * 2 * 8, (size_t)nx * 8, (size_t)nx * 8,
                            (size_t)GLUE_NVEC * nv * 4, (size_t)2 * GLUE_HIST * nv * 4};
  void* ptr[14];
  const bool ok = arena_take(ar, 14, sizes, ptr, &s) == 0;
  if (ok) {
    d_off = (int64_t*)ptr[0];
    d_geo = (double*)ptr[1];
    d_x0 = (float*)ptr[2];
    d_tgt = (float*)ptr[3];
    d_grid = (int32_t*)ptr[4];
    d_prior = (float*)ptr[5];
    d_kcnt = (int32_t*)ptr[6];
    d_xout = (float*)ptr[7];
    d_stats = (int32_t*)ptr[8];
    d_loss = (double*)ptr[9];
    P.X = (double*)ptr[10];
    P.AX = (double*)ptr[11];
    P.V = (float*)ptr[12];
    P.H = (float*)ptr[13];
  }
  if (!ok) {
    rc = GEOBPE_EHIP;
  } else {
    hipMemcpyAsync(d_off, h_res_off, (S + 1) * 8, hipMemcpyHostToDevice, s);
    hipMemcpyAsync(d_geo, h_geo, R * 9 * 8, hipMemcpyHostToDevice, s);
    hipMemcpyAsync(d_x0, h_x0, G * 3 * 4, hipMemcpyHostToDevice, s);
    hipMemcpyAsync(d_tgt, h_tgt, G * 12 * 4, hipMemcpyHostToDevice, s);
    hipMemcpyAsync(d_grid, h_grid, S * 4, hipMemcpyHostToDevice, s);
    hipMemcpyAsync(d_prior, h_prior, (int64_t)n_grid * 6 * kmax * 4, hipMemcpyHostToDevice, s);
    hipMemcpyAsync(d_kcnt, h_kcnt, (int64_t)n_grid * 3 * 4, hipMemcpyHostToDevice, s);
    P.roff = d_off;
    P.geo = d_geo;
    P.tgt = d_tgt;
    P.grid = d_grid;
    P.prior = d_prior;
    P.kcnt = d_kcnt;
    if (wave) {
      GlueWaveProb W{};
      W.roff = d_off;
      W.geo = d_geo;
      W.tgt = d_tgt;
      W.grid = d_grid;
      W.prior = d_prior;
      W.kcnt = d_kcnt;
      W.kmax = kmax;
      W.lam = lam;
      W.wR = w_rot;
      W.wt = w_trans;
      W.X = P.X;
      W.AX = P.AX;
      W.V = P.V;
      W.H = P.H;
      W.NG = NG;
      hipLaunchKernelGGL(k_glue_wave, dim3((unsigned)S), dim3(GW), 0, s, W, S, (const float*)d_x0, d_xout, d_stats,
                         d_loss);
    } else {
      hipLaunchKernelGGL(k_glue_opt, dim3((unsigned)((S + 63) / 64)), dim3(64), 0, s, P, (const float*)d_x0, d_xout,
                         d_stats, d_loss);
    }
    if (hipGetLastError() != hipSuccess) rc = GEOBPE_EHIP;
    if (!rc && (hipMemcpyAsync(h_xout, d_xout, G * 3 * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipMemcpyAsync(h_stats, d_stats, S * 2 * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipMemcpyAsync(h_loss, d_loss, S * 2 * 8, hipMemcpyDeviceToHost, s) != hipSuccess))
      rc = GEOBPE_EHIP;
    if (hipStreamSynchronize(s) != hipSuccess) rc = GEOBPE_EHIP;
  }
  return rc;
}

int geobpe_set_record_events(geobpe_ctx* c, int on) {
  if (!c) return GEOBPE_EARG;
  HIPCHK(c, hipSetDevice(c->device));
  if (!on) {
    if (c->ev) {
      HIPCHK(c, hipStreamSynchronize(c->stream));
      hipFree(c->ev);
      hipFree(c->ev_n);
    }
    c->ev = nullptr;
    c->ev_n = nullptr;
    c->ev_cap = 0;
    c->D.ev = nullptr;
    c->D.ev_n = nullptr;
    c->D.ev_cap = 0;
    return 0;
  }
  if (c->ev) return 0;
  if (c->h_state && c->h_state->iter > 0) return fail(c, GEOBPE_EARG, "record events before the first merge");
  c->ev_cap = std::max<int64_t>(c->R, 1);  // every merge removes one token: < R events in all
  HIPCHK(c, hipMalloc(&c->ev, (size_t)c->ev_cap * sizeof(int4)));
  HIPCHK(c, hipMalloc(&c->ev_n, sizeof(unsigned long long)));
  HIPCHK(c, hipMemsetAsync(c->ev_n, 0, sizeof(unsigned long long), c->stream));
  c->D.ev = c->ev;  // (k_tail writes its merges' events itself)
  c->D.ev_cap = c->ev_cap;
  c->D.ev_n = c->ev_n;
  return 0;
}

int64_t geobpe_events(geobpe_ctx* c, int32_t* h_merge, int32_t* h_a, int32_t* h_b) {
  if (!c || !c->ev) return -1;
  if (sync_state(c)) return -1;
  unsigned long long n = 0;
  if (hipMemcpy(&n, c->ev_n, sizeof n, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if ((int64_t)n > c->ev_cap) {
    fail(c, GEOBPE_ECAPACITY, "merge-event log overflow (%llu > %lld)", n, (long long)c->ev_cap);
    return -1;
  }
  if (h_merge && h_a && h_b && n) {
    std::vector<int4> ev(n);
    if (hipMemcpy(ev.data(), c->ev, n * sizeof(int4), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    for (size_t i = 0; i < n; i++) {
      h_merge[i] = ev[i].x;
      h_a[i] = ev[i].y;
      h_b[i] = ev[i].z;
    }
  }
  return (int64_t)n;
}

int geobpe_synchronize(geobpe_ctx* c) {
  if (!c) return GEOBPE_EARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return sync_state(c);
}

// ---------------------------------------------------------------- the engine's own exchange
static thread_local std::string g_comm_err;

const char* geobpe_comm_error(void) { return g_comm_err.c_str(); }

static int rccl_load(const char* path, RcclApi& a, std::string& err) {
  if (a.h) return 0;
  void* h = dlopen(path && *path ? path : "librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    err = std::string("dlopen RCCL: ") + dlerror();
    return GEOBPE_EARG;
  }
  a.GetUniqueId = (decltype(a.GetUniqueId))dlsym(h, "ncclGetUniqueId");
  a.CommInitRank = (decltype(a.CommInitRank))dlsym(h, "ncclCommInitRank");
  a.AllGather = (decltype(a.AllGather))dlsym(h, "ncclAllGather");
  a.CommDestroy = (decltype(a.CommDestroy))dlsym(h, "ncclCommDestroy");
  a.GetErrorString = (decltype(a.GetErrorString))dlsym(h, "ncclGetErrorString");
  if (!a.GetUniqueId || !a.CommInitRank || !a.AllGather || !a.CommDestroy) {
    err = "RCCL library lacks ncclGetUniqueId / ncclCommInitRank / ncclAllGather / ncclCommDestroy";
    return GEOBPE_EARG;
  }
  a.h = h;
  return 0;
}

int geobpe_comm_unique_id(const char* rccl_path, void* out128) {
  if (!out128) return GEOBPE_EARG;
  static RcclApi api;
  g_comm_err.clear();
  int rc;
  if ((rc = rccl_load(rccl_path, api, g_comm_err))) return rc;
  ncclUniqueId id;
  const ncclResult_t r = api.GetUniqueId(&id);
  if (r != ncclSuccess) {
    g_comm_err = std::string("ncclGetUniqueId: ") + (api.GetErrorString ? api.GetErrorString(r) : "?");
    return GEOBPE_EHIP;
  }
  memcpy(out128, &id, sizeof id);
  return 0;
}

int geobpe_comm_init_rccl(geobpe_ctx* c, const char* rccl_path, const void* unique_id, int32_t nranks, int32_t rank) {
  if (!c || !unique_id || nranks < 1 || rank < 0 || rank >= nranks || nranks > PIPE_MAX_WORLD) return GEOBPE_EARG;
  if (c->x_kind) return fail(c, GEOBPE_EARG, "exchange already set up");
  std::string err;
  if (rccl_load(rccl_path, c->rccl, err)) return fail(c, GEOBPE_EARG, "%s", err.c_str());
  HIPCHK(c, hipSetDevice(c->device));
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof id);
  const ncclResult_t r = c->rccl.CommInitRank(&c->comm, nranks, id, rank);
  if (r != ncclSuccess)
    return fail(c, GEOBPE_EHIP, "ncclCommInitRank: %s", c->rccl.GetErrorString ? c->rccl.GetErrorString(r) : "?");
  c->x_kind = 1;
  c->x_world = nranks;
  c->x_rank = rank;
  return 0;
}

int geobpe_comm_set_callback(geobpe_ctx* c, geobpe_allgather_fn fn, void* user, int32_t nranks, int32_t rank) {
  if (!c || !fn || nranks < 1 || rank < 0 || rank >= nranks || nranks > PIPE_MAX_WORLD) return GEOBPE_EARG;
  if (c->x_kind) return fail(c, GEOBPE_EARG, "exchange already set up");
  c->x_kind = 2;
  c->x_fn = fn;
  c->x_user = user;
  c->x_world = nranks;
  c->x_rank = rank;
  return 0;
}

int geobpe_comm_set_slot(geobpe_ctx* c, int64_t records) {
  if (!c || records < 0) return GEOBPE_EARG;
  c->x_fixed = records;  // 0: sized from the last import (2x the largest, a power of two, 1024..65536)
  return 0;
}

int geobpe_set_collapse(geobpe_ctx* c, int on) {
  if (!c) return GEOBPE_EARG;
  if (c->collapsed && !on) return fail(c, GEOBPE_EARG, "the engine has collapsed already");
  c->collapse_on = on != 0;
  return 0;
}

int geobpe_collapsed(geobpe_ctx* c) { return c && c->collapsed ? 1 : 0; }

int geobpe_comm_peer(geobpe_ctx* c, int on) {
  if (!c) return GEOBPE_EARG;
  if (c->x_peer_ready && !on) return fail(c, GEOBPE_EARG, "the peer exchange is set up already");
  c->x_peer_want = on != 0;
  return 0;
}

int geobpe_comm_peer_active(geobpe_ctx* c) { return c && c->x_peer_ready ? 1 : 0; }

namespace {

int grow_dev(geobpe_ctx* c, uint8_t** p, int64_t* have, int64_t bytes) {
  if (*have >= bytes) return 0;
  if (*p) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(*p);
    *p = nullptr;
  }
  HIPCHK(c, hipMalloc((void**)p, (size_t)std::max<int64_t>(bytes, 64)));
  *have = bytes;
  return 0;
}

// every rank's `bytes` from d_send, rank-major into d_recv (world * bytes), stream-ordered
// for RCCL; through pinned host staging and the caller's collective for the callback
int x_allgather(geobpe_ctx* c, const void* d_send, void* d_recv, int64_t bytes) {
  if (bytes <= 0) return 0;
  if (c->x_kind == 1) {
    const ncclResult_t r = c->rccl.AllGather(d_send, d_recv, (size_t)bytes, ncclUint8, c->comm, c->stream);
    if (r != ncclSuccess)
      return fail(c, GEOBPE_EHIP, "ncclAllGather: %s", c->rccl.GetErrorString ? c->rccl.GetErrorString(r) : "?");
    return 0;
  }
  const int64_t need = bytes * c->x_world;
  if (c->x_hbytes < need) {
    HIPCHK(c, hipStreamSynchronize(c->stream));  // (the last copy out of x_hrecv may be in flight)
    if (c->x_hsend) hipHostFree(c->x_hsend);
    if (c->x_hrecv) hipHostFree(c->x_hrecv);
    HIPCHK(c, hipHostMalloc((void**)&c->x_hsend, (size_t)need, hipHostMallocDefault));
    HIPCHK(c, hipHostMalloc((void**)&c->x_hrecv, (size_t)need, hipHostMallocDefault));
    c->x_hbytes = need;
  }
  HIPCHK(c, hipMemcpyAsync(c->x_hsend, d_send, (size_t)bytes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->x_fn(c->x_user, c->x_hsend, c->x_hrecv, bytes) != 0) return fail(c, GEOBPE_EHIP, "exchange callback failed");
  HIPCHK(c, hipMemcpyAsync(d_recv, c->x_hrecv, (size_t)need, hipMemcpyHostToDevice, c->stream));
  return 0;
}

// the stalled merge: every rank's full record list (counts from the slot headers, then
// records sized by the largest), compacted rank by rank, imported on every rank
int x_resolve(geobpe_ctx* c) {
  const int64_t REC = (int64_t)sizeof(DeltaRec), W = c->x_world;
  int rc;
  if ((rc = grow_dev(c, &c->x_tmp, &c->x_tmp_bytes, 8 * W))) return rc;
  if ((rc = x_allgather(c, c->x_pbuf, c->x_tmp, 8))) return rc;
  std::vector<int64_t> cnt(W);
  HIPCHK(c, hipMemcpyAsync(cnt.data(), c->x_tmp, 8 * W, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const int64_t m = *std::max_element(cnt.begin(), cnt.end());
  if (m > c->x_pcap) return fail(c, GEOBPE_ECAPACITY, "delta export needs %lld records (cap %lld)", (long long)m,
                                 (long long)c->x_pcap);
  int64_t total = 0;
  for (int64_t r : cnt) total += r;
  if ((rc = grow_dev(c, &c->x_tmp, &c->x_tmp_bytes, std::max<int64_t>(8 * W, W * m * REC))) ||
      (rc = grow_dev(c, &c->x_flat, &c->x_flat_bytes, std::max<int64_t>(total, 1) * REC)))
    return rc;
  if ((rc = x_allgather(c, c->x_pbuf + REC, c->x_tmp, m * REC))) return rc;
  int64_t off = 0;
  for (int64_t r = 0; r < W; r++) {
    if (c->x_peer_ready && !c->x_loop && r == c->x_rank) continue;  // (the peer exchange applied this rank's own already)
    if (cnt[r])
      HIPCHK(c, hipMemcpyAsync(c->x_flat + off * REC, c->x_tmp + r * m * REC, cnt[r] * REC, hipMemcpyDeviceToDevice,
                               c->stream));
    off += cnt[r];
  }
  return geobpe_pipeline_resolve(c, c->x_flat, off);
}

// every rank's `bytes` of host data, rank-major, through the exchange (device staging)
int x_allgather_host(geobpe_ctx* c, const void* h_send, int64_t bytes, std::vector<uint8_t>& h_recv) {
  const int64_t W = c->x_world;
  int rc;
  if ((rc = grow_dev(c, &c->x_flat, &c->x_flat_bytes, bytes)) ||
      (rc = grow_dev(c, &c->x_tmp, &c->x_tmp_bytes, W * bytes)))
    return rc;
  HIPCHK(c, hipMemcpyAsync(c->x_flat, h_send, (size_t)bytes, hipMemcpyHostToDevice, c->stream));
  if ((rc = x_allgather(c, c->x_flat, c->x_tmp, bytes))) return rc;
  h_recv.resize((size_t)(W * bytes));
  HIPCHK(c, hipMemcpyAsync(h_recv.data(), c->x_tmp, (size_t)(W * bytes), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

// every rank's block of n[r] elements of `per` bytes (d_src: this rank's) into d_dst at the
// rank's element base: one all-gather of blocks padded to the largest
int x_gather_blocks(geobpe_ctx* c, const void* d_src, void* d_dst, const std::vector<int64_t>& n,
                    const std::vector<int64_t>& base, int64_t per) {
  const int64_t W = c->x_world;
  const int64_t nmax = *std::max_element(n.begin(), n.end());
  int rc;
  if ((rc = grow_dev(c, &c->x_flat, &c->x_flat_bytes, std::max<int64_t>(nmax * per, 8))) ||
      (rc = grow_dev(c, &c->x_tmp, &c->x_tmp_bytes, std::max<int64_t>(W * nmax * per, 8))))
    return rc;
  if (n[c->x_rank]) HIPCHK(c, hipMemcpyAsync(c->x_flat, d_src, (size_t)(n[c->x_rank] * per), hipMemcpyDeviceToDevice, c->stream));
  if ((rc = x_allgather(c, c->x_flat, c->x_tmp, nmax * per))) return rc;
  for (int64_t r = 0; r < W; r++)
    if (n[r])
      HIPCHK(c, hipMemcpyAsync((uint8_t*)d_dst + base[r] * per, c->x_tmp + r * nmax * per, (size_t)(n[r] * per),
                               hipMemcpyDeviceToDevice, c->stream));
  return 0;
}

// every rank's yes: a collective every rank reaches (the decisions that lead here read only
// replicated data), so a rank that cannot go on says so instead of leaving its peers blocked in
// the next collective (the collapse's allocations could fail between gathers)
int x_agree(geobpe_ctx* c, bool mine, bool* all) {
  const int32_t v = mine ? 1 : 0;
  std::vector<uint8_t> raw;
  int rc;
  if ((rc = x_allgather_host(c, &v, 4, raw))) return rc;
  *all = true;
  for (int64_t r = 0; r < c->x_world; r++) *all = *all && reinterpret_cast<const int32_t*>(raw.data())[r] != 0;
  return 0;
}

// device memory still free, less a margin for the runtime and RCCL
bool x_fits(int64_t bytes) {
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) return false;
  return (int64_t)fr - bytes > (int64_t)(1LL << 30);
}

// The peer exchange (exchange.h), once per engine: this rank's receive area (2 parities x W
// slots of XHDR + capf records), its IPC handle all-gathered, every other rank's area opened
// here (same node: xGMI peer memory; ranks sharing a GPU: the same device).  Every rank's yes is
// agreed on; a rank that cannot map every peer turns the peer exchange off on every rank (the
// all-gather exchange stays).  capf: the fixed slot size when geobpe_comm_set_slot set one (tests
// force stalls with tiny slots), else the all-gather path's largest (65 536 records).
int x_peer_setup(geobpe_ctx* c, int64_t capf) {
  if (c->x_peer_ready || !c->x_peer_want) return 0;
  // (records per slot: the all-gather path's 65 536 made the heaviest C3 merges stall at world 1;
  // 2^19 x 40 B x 2 parities x 8 ranks = 336 MB of the 288 GB)
  const int64_t W = c->x_world, me = c->x_rank;
  int rc;
  bool ok = W >= 1 && W <= XPEER_MAX;
  c->x_rcapf = capf;
  c->x_slot = ((XHDR + capf * (int64_t)sizeof(DeltaRec)) + 255) / 256 * 256;
  hipIpcMemHandle_t mine;
  memset(&mine, 0, sizeof mine);
  if (ok) ok = hipMalloc((void**)&c->x_recv, (size_t)(2 * W * c->x_slot)) == hipSuccess;
  c->x_chkcap = (W * capf + c->nba - 2) / std::max(1, c->nba - 1) + 64;  // (one import share of every rank's slot)
  if (ok) ok = !dalloc(c, &c->x_chk, 2 * (int64_t)c->nba * c->x_chkcap) && !dalloc(c, &c->x_chkcnt, 2 * c->nba, 0);  // (two halves, exchange.h)
  if (ok) ok = hipMemsetAsync(c->x_recv, 0, (size_t)(2 * W * c->x_slot), c->stream) == hipSuccess &&
               hipStreamSynchronize(c->stream) == hipSuccess;
  if (ok && W > 1) ok = hipIpcGetMemHandle(&mine, c->x_recv) == hipSuccess;
  if (W > 1) {  // every rank's {ok, handle}; a handle is opened only when every rank made one
    struct {
      int64_t ok;
      hipIpcMemHandle_t h;
    } rec;
    rec.ok = ok ? 1 : 0;
    rec.h = mine;
    std::vector<uint8_t> all;
    if ((rc = x_allgather_host(c, &rec, sizeof rec, all))) return rc;
    for (int64_t q = 0; q < W; q++) ok = ok && reinterpret_cast<const decltype(rec)*>(all.data())[q].ok != 0;
    for (int64_t q = 0; q < W && ok; q++) {
      if (q == me) continue;
      void* p = nullptr;
      ok = hipIpcOpenMemHandle(&p, reinterpret_cast<const decltype(rec)*>(all.data())[q].h,
                               hipIpcMemLazyEnablePeerAccess) == hipSuccess;
      c->x_peers[q] = (uint8_t*)p;
    }
  }
  int can = 0;
  c->x_cpwait = hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, c->device) == hipSuccess && can;
  // (the stream waits on the command processor for ONE peer; with more, one waiter kernel: each
  // hipStreamWaitValue32 costs the host ~2.8 us to enqueue, probe tools/probe/waitvalue.hip --
  // at 7 peers more than a merge's kernels take on the device)
  c->x_cpwait = c->x_cpwait && W == 2;
  if (const char* e = getenv("GEOBPE_PEER_WAIT")) c->x_cpwait = atoi(e) != 0;  // (1: command processor, 0: waiter kernel)
  bool every = ok;
  if (W > 1 && (rc = x_agree(c, ok, &every))) return rc;
  if (!every) {
    for (int64_t q = 0; q < W; q++)
      if (q != me && c->x_peers[q]) hipIpcCloseMemHandle(c->x_peers[q]);
    if (c->x_recv) hipFree(c->x_recv);
    c->x_recv = nullptr;
    dfree(c, &c->x_chk);
    dfree(c, &c->x_chkcnt);
    for (auto& p : c->x_peers) p = nullptr;
    c->x_peer_want = false;
    return 0;
  }
  c->x_peers[me] = c->x_recv;
  // (loopback rehearsal, one rank: its records go to its own slot and are imported by content
  // hash, as a peer's -- the import cost a rank of N pays, measured on one GPU)
  if (const char* e = getenv("GEOBPE_PEER_LOOPBACK")) c->x_loop = W == 1 && atoi(e) != 0;
  c->x_hseq = 1;
  c->x_prev_seq = 0;
  c->x_pending = false;
  c->x_peer_ready = true;
  return 0;
}

// Before the first pipelined merge: what a collapse moves that never changes after
// initialize() -- every rank's junction symbols (int32 and 16-bit copies) and row offsets -- is
// gathered once, off the switch (the collapse then moves only the 16-B token
// records).  Every step that can fail on one rank (the sizes, the allocations) is agreed on by
// every rank before the gathers; a rank that cannot hold them turns the collapse off on all.
int x_collapse_prepare(geobpe_ctx* c) {
  if (c->cg_ready || !c->collapse_on) return 0;
  const int64_t W = c->x_world, me = c->x_rank;
  int rc;
  const int64_t mine[3] = {c->R, c->nrows, c->Lmax};
  std::vector<uint8_t> raw;
  if ((rc = x_allgather_host(c, mine, sizeof mine, raw))) return rc;
  const int64_t* all = reinterpret_cast<const int64_t*>(raw.data());
  c->cg_nR.assign(W, 0);
  c->cg_nN.assign(W, 0);
  c->cg_bR.assign(W + 1, 0);
  c->cg_bN.assign(W + 1, 0);
  c->cg_Lmax = 1;
  for (int64_t r = 0; r < W; r++) {
    c->cg_nR[r] = all[3 * r];
    c->cg_nN[r] = all[3 * r + 1];
    c->cg_Lmax = std::max(c->cg_Lmax, all[3 * r + 2]);
    c->cg_bR[r + 1] = c->cg_bR[r] + c->cg_nR[r];
    c->cg_bN[r + 1] = c->cg_bN[r] + c->cg_nN[r];
  }
  const int64_t Rt = c->cg_bR[W], Nt = c->cg_bN[W];
  const int64_t nmax = *std::max_element(c->cg_nR.begin(), c->cg_nR.end());
  const int64_t per = c->D.gs16 ? 6 : 4;
  bool ok = c->cg_nR[me] == c->R && c->cg_nN[me] == c->nrows && Rt < INT32_MAX / 4 &&
            x_fits(Rt * per + (Nt + 1) * 8 + (W + 1) * nmax * 4 + 16 * Rt + tail_bytes(c, Rt));
  Dev& D = c->D;
  if (ok) ok = !dalloc(c, &c->cg_gsym, Rt + 8, 0) && !dalloc(c, &c->cg_row, Nt + 1) &&
               !(D.gs16 && dalloc(c, &c->cg_gs16, Rt + 8, 0xFF)) &&
               !grow_dev(c, &c->x_flat, &c->x_flat_bytes, std::max<int64_t>(nmax * 4, 8)) &&
               !grow_dev(c, &c->x_tmp, &c->x_tmp_bytes, std::max<int64_t>(W * nmax * 4, 8));
  bool every = false;
  if ((rc = x_agree(c, ok, &every))) return rc;
  if (!every) {  // (consistent on every rank: the sharded middle regime instead)
    dfree(c, &c->cg_gsym);
    dfree(c, &c->cg_row);
    if (c->cg_gs16) dfree(c, &c->cg_gs16);
    c->collapse_on = false;
    return 0;
  }
  if ((rc = x_gather_blocks(c, D.gsym, c->cg_gsym, c->cg_nR, c->cg_bR, sizeof(int32_t))) ||
      (D.gs16 && (rc = x_gather_blocks(c, D.gs16, c->cg_gs16, c->cg_nR, c->cg_bR, sizeof(uint16_t)))))
    return rc;
  // row offsets: every rank's (local, then moved to its residue base), the total at the end
  const int64_t nNmax = *std::max_element(c->cg_nN.begin(), c->cg_nN.end());
  std::vector<int64_t> send(std::max<int64_t>(nNmax, 1), 0);
  std::copy(c->row_off.begin(), c->row_off.begin() + c->nrows, send.begin());
  if ((rc = x_allgather_host(c, send.data(), (int64_t)send.size() * 8, raw))) return rc;
  const int64_t* ro = reinterpret_cast<const int64_t*>(raw.data());
  c->cg_rows.assign(Nt + 1, 0);
  for (int64_t r = 0; r < W; r++)
    for (int64_t i = 0; i < c->cg_nN[r]; i++) c->cg_rows[c->cg_bN[r] + i] = c->cg_bR[r] + ro[r * (int64_t)send.size() + i];
  c->cg_rows[Nt] = Rt;
  HIPCHK(c, hipMemcpyAsync(c->cg_row, c->cg_rows.data(), (Nt + 1) * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->cg_ready = true;
  return 0;
}

// the collapse as a cost decision: it pays once -- the token records' all-gather
// (16 B a residue at ~200 GB/s per rank over xGMI), the re-keying pass (~0.5 ms) and the
// whole-corpus list build (~1.5 ms) at C3's 30 M residues, ~0.2 ms of synchronisations and
// launches -- and saves the exchange of every later merge of the run (~25 us a merge: the
// record export, the all-gather and the import of the world-1 rehearsal), so it is
// taken when the run has enough merges left to earn it back (C3: ~190)
bool x_collapse_pays(const geobpe_ctx* c, int64_t left) {
  if (!c->cg_ready || c->cg_bR.empty()) return false;
  const double Rt = (double)c->cg_bR.back();
  const double cost_us = 200.0 + Rt * (16.0 / 200e3 + 2.0e3 / 30e6);
  return (double)left * (c->x_peer_ready ? 10.0 : 25.0) > cost_us;  // (the peer exchange's ~10 us a merge)
}

// The middle-regime switch of the row-sharded loop: stop sharding.  Below mid_thresh
// occurrences a merge is a fixed chain of dependent round trips whatever a rank holds, so
// the per-merge exchange (all-gather + import) is pure overhead there (N > 1
// slower than N = 1 in that regime).  Every rank gathers every rank's token records once (the
// junction symbols and row offsets were gathered before the loop, x_collapse_prepare), re-keys
// the foreign blocks' pairs in its own key table (k_collapse_fix) and continues as the one-rank
// loop over the whole corpus -- every rank making the same merges with no exchange, its own
// rows a window of the whole.  The counts need no change: they were global (replicated)
// already.  Called at a poll of geobpe_run_exchange, after geobpe_pipeline_end (nothing in
// flight, nothing stalled).  Every allocation comes first and every rank agrees before the
// gather (x_agree): *done = false on every rank when one of them cannot take the whole corpus,
// and the loop goes on sharded.
int x_collapse(geobpe_ctx* c, bool* done) {
  *done = false;
  if (!c->cg_ready) return 0;
  const int64_t W = c->x_world, me = c->x_rank;
  int rc;
  if ((rc = sync_state(c))) return rc;  // (flushes the last merge's place)
  Dev& D = c->D;
  const int64_t Rt = c->cg_bR[W], Nt = c->cg_bN[W], Lmax = c->cg_Lmax;
  const int64_t nmax = *std::max_element(c->cg_nR.begin(), c->cg_nR.end());
  int4* tok2 = nullptr;
  int64_t* d_base = nullptr;
  u64 *dp1 = nullptr, *dp2 = nullptr;
  const int64_t pwn = 2 * Lmax + 8;
  bool ok = x_fits(16 * Rt + 2 * W * nmax * 16 + tail_bytes(c, Rt)) && !dalloc(c, &tok2, Rt + 8, 0xFF) &&
            !dalloc(c, &d_base, W + 1) &&
            (Lmax <= c->Lmax || (!dalloc(c, &dp1, pwn) && !dalloc(c, &dp2, pwn))) &&
            !grow_dev(c, &c->x_flat, &c->x_flat_bytes, std::max<int64_t>(nmax * 16, 8)) &&
            !grow_dev(c, &c->x_tmp, &c->x_tmp_bytes, std::max<int64_t>(W * nmax * 16, 8));
  bool every = false;
  if ((rc = x_agree(c, ok, &every))) return rc;
  if (!every) {  // (declined for good: the whole-corpus static arrays of x_collapse_prepare go too)
    dfree(c, &tok2);
    dfree(c, &d_base);
    if (dp1) dfree(c, &dp1);
    if (dp2) dfree(c, &dp2);
    dfree(c, &c->cg_gsym);
    dfree(c, &c->cg_row);
    if (c->cg_gs16) dfree(c, &c->cg_gs16);
    c->cg_ready = false;
    c->collapse_on = false;
    return 0;
  }
  if ((rc = x_gather_blocks(c, D.tok, tok2, c->cg_nR, c->cg_bR, sizeof(int4)))) return rc;
  // the longest chain anywhere bounds the token lengths the content hashes combine
  if (Lmax > c->Lmax) {
    std::vector<u64> p1(pwn), p2(pwn);
    p1[0] = p2[0] = 1;
    for (int64_t i = 1; i < pwn; i++) {
      p1[i] = mulmod61(p1[i - 1], HP1);
      p2[i] = mulmod61(p2[i - 1], HP2);
    }
    HIPCHK(c, hipMemcpyAsync(dp1, p1.data(), pwn * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(dp2, p2.data(), pwn * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));  // (the host vectors go out of scope)
    D.pw1 = dp1;
    D.pw2 = dp2;
    D.pwn = pwn;
    c->Lmax = Lmax;
  }
  // the whole corpus from here on
  dfree(c, &D.tok);
  dfree(c, &D.gsym);
  if (D.gs16) dfree(c, &D.gs16);
  dfree(c, &c->d_row_off);
  D.tok = tok2;
  D.gsym = c->cg_gsym;
  D.gs16 = c->cg_gs16;
  c->d_row_off = c->cg_row;
  D.row_off = c->cg_row;
  c->cg_gsym = nullptr;
  c->cg_gs16 = nullptr;
  c->cg_row = nullptr;
  c->row_off = c->cg_rows;
  c->own_row0 = c->cg_bN[me];
  c->own_row1 = c->cg_bN[me + 1];
  c->R = Rt;
  D.R = Rt;
  c->nrows = Nt;
  D.nrows = Nt;
  HIPCHK(c, hipMemcpyAsync(d_base, c->cg_bR.data(), (W + 1) * 8, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(k_collapse_fix, dim3(c->nb), dim3(BLOCK), 0, c->stream, c->D, (const int64_t*)d_base, (int)W,
                     (int)me);
  HIPCHK(c, hipGetLastError());
  if ((rc = sync_state(c))) return rc;
  dfree(c, &d_base);
  // the per-key lists and the middle regime's buffers are sized by the residues: made again
  if (c->tail_ready) {
    dfree(c, &D.kpool);
    dfree(c, &D.TM);
    dfree(c, &D.TH);
    dfree(c, &D.TS);
    dfree(c, &D.TR);
    dfree(c, &D.TK);
    c->tail_ready = false;
  }
  c->h_state->kp_valid = 0;
  HIPCHK(c, hipMemsetAsync(&D.st->kp_valid, 0, 4, c->stream));
  c->distributed = false;
  c->collapsed = true;
  c->mid_on = true;
  *done = true;
  return 0;
}

}  // namespace

// the pipelined N > 1 loop with the engine's own exchange (TorchGroup.run_pipelined in C++):
// per iteration select / find / commit and the slot export, ONE all-gather of the fixed
// slots on the engine's stream, the import; a poll every few iterations (the window doubles
// up to 64, back to 1 after a stall), a stalled merge re-exchanged in full.  Every rank sees
// the same polls, so every rank issues the same collectives.
}  // extern "C"
namespace {
// the pinned merge-log mirror grown to hold records [0, need) (geobpe_run_log's)
int grow_h_log(geobpe_ctx* c, int64_t need) {
  need = std::min<int64_t>(c->D.KC, need);
  if (need <= c->h_log_cap) return 0;
  const int64_t cap = std::min<int64_t>(c->D.KC, std::max<int64_t>({need, 2 * c->h_log_cap, 4096}));
  LogRec* p = nullptr;
  HIPCHK(c, hipHostMalloc((void**)&p, (size_t)cap * sizeof(LogRec), hipHostMallocDefault));
  if (c->h_log) {
    memcpy(p, c->h_log, (size_t)c->h_log_cap * sizeof(LogRec));
    hipHostFree(c->h_log);
  }
  c->h_log = p;
  c->h_log_cap = cap;
  return 0;
}
int run_exchange_impl(geobpe_ctx* c, int64_t n_merges, int64_t* n_done, int64_t* log_first);
}  // namespace
extern "C" {

int geobpe_run_exchange(geobpe_ctx* c, int64_t n_merges, int64_t* n_done) {
  return run_exchange_impl(c, n_merges, n_done, nullptr);
}

// geobpe_run_exchange with the run's merge records ({new id, count, merged} per merge, as
// geobpe_run_log) pulled inside its last synchronisation; *first = the first merge's index, or -1
// when the run ended in the one-rank loop (a collapse: then geobpe_merge_log has them)
int geobpe_run_exchange_log(geobpe_ctx* c, int64_t n_merges, int64_t* n_done, int64_t* first, int64_t* h_out,
                            int64_t cap) {
  if (!c || !first || !n_done || (cap > 0 && !h_out)) return GEOBPE_EARG;
  int rc = run_exchange_impl(c, n_merges, n_done, first);
  if (rc || *first < 0) return rc;
  const int64_t n = std::min(*n_done, cap);
  for (int64_t i = 0; i < n; i++) {
    const LogRec& r = c->h_log[*first + i];
    h_out[3 * i] = r.nid;
    h_out[3 * i + 1] = r.count;
    h_out[3 * i + 2] = r.nmerged;
  }
  return 0;
}

}  // extern "C"
namespace {
int run_exchange_impl(geobpe_ctx* c, int64_t n_merges, int64_t* n_done, int64_t* log_first) {
  static const bool xt = getenv("GEOBPE_XTIME") != nullptr;  // (host phase times to stderr: diagnostics)
  auto now_us = []() { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double xt0 = xt ? now_us() : 0;
  if (log_first) *log_first = -1;
  if (!c || n_merges < 0) return GEOBPE_EARG;
  if (c->collapsed) return geobpe_run(c, n_merges, n_done);  // (every rank holds the whole corpus)
  if (!c->distributed || !c->keys_ready) return fail(c, GEOBPE_EARG, "run_exchange needs a distributed, binned engine");
  if (!c->x_kind) return fail(c, GEOBPE_EARG, "no exchange set up (geobpe_comm_init_rccl / geobpe_comm_set_callback)");
  HIPCHK(c, hipSetDevice(c->device));
  const int64_t REC = (int64_t)sizeof(DeltaRec), W = c->x_world;
  constexpr int64_t CAP_MIN = 1024, CAP_MAX = 65536, AHEAD_MAX = 64;
  int rc;
  if (!c->x_pbuf) {
    c->x_pcap = 3 * c->R + 65536;
    HIPCHK(c, hipMalloc((void**)&c->x_pbuf, (size_t)((1 + c->x_pcap) * REC)));
    HIPCHK(c, hipMemsetAsync(c->x_pbuf, 0, (size_t)((1 + c->x_pcap) * REC), c->stream));
  }
  // the gathered slots: W x the largest slot this run can use (geobpe_comm_set_slot may have
  // raised the fixed size since the last run)
  if ((rc = grow_dev(c, &c->x_gath, &c->x_gath_bytes, W * (1 + std::max(CAP_MAX, c->x_fixed)) * REC))) return rc;
  if (!c->ev && (rc = x_collapse_prepare(c))) return rc;  // (once: the collapse's static arrays)
  // (once: the peer exchange, unless GEOBPE_PEER=0 or more ranks than one node holds)
  if (const char* e = getenv("GEOBPE_PEER")) c->x_peer_want = c->x_peer_want && atoi(e) != 0;
  if (W > XPEER_MAX) c->x_peer_want = false;
  if ((rc = x_peer_setup(c, c->x_fixed ? c->x_fixed : (int64_t)1 << 19))) return rc;
  const bool peer = c->x_peer_ready;
  // the regimes of the sharded loop: a rank runs the middle regime once ITS share of
  // the winner's occurrences (count / W) is below the one-rank threshold, and the ranks collapse
  // into the one-rank loop only below x_collapse_at, where one rank's late merge costs about what
  // a sharded merge plus its exchange does.  Both read only replicated data (the winner's global
  // count), so every rank switches at the same poll.
  // A sharded rank switches at 1.5x the one-rank threshold of its share: its full-grid merges pay
  // the exchange per key record, and the measured crossover of the two regimes moves up (DESIGN 5:
  // one rank's share of a 2-way run, 50-85 k occurrences, middle regime 93.5 vs full grid 94.0 us a
  // merge with the exchange, 60 vs 70 without).  A world-1 rehearsal of one rank's share of an
  // N-way run (x_shards = N) takes N's thresholds: its counts are the share's, the run's are N x.
  // Two ranks stay in the full grid down to the collapse: there their middle regime does not beat it
  // (93.5 vs 94.0 us), and the shard's list build (~1.3 ms at half of C3) would be paid again by
  // the collapse's for the whole corpus.
  const bool sharded = W > 1 || c->x_shards > 1;
  const int64_t collapse_at = (peer ? c->x_collapse_at : c->mid_thresh) / (W > 1 ? 1 : c->x_shards);  // (the all-gather's ~30 us a merge: sooner)
  const int64_t mid_at = (W == 2 || c->x_shards == 2) && c->collapse_on
                             ? collapse_at
                             : (sharded ? c->mid_thresh * 3 / 2 : c->mid_thresh) * W;
  if (!c->x_hlog) HIPCHK(c, hipHostMalloc((void**)&c->x_hlog, (size_t)(AHEAD_MAX + 2) * sizeof(LogRec), hipHostMallocDefault));
  const double xt1 = xt ? now_us() : 0;
  if ((rc = pipeline_begin_impl(c, true))) return rc;
  if (xt) fprintf(stderr, "xtime: preamble %.1f us, begin %.1f us (lite %d)\n", xt1 - xt0, now_us() - xt1,
                  (int)(c->enq == c->enq_synced));
  int64_t out[4];
  int64_t done = 0;
  if (!peer) rc = geobpe_pipeline_poll(c, out);  // (the slot sizing's largest count starts again)
  const int64_t it0 = c->h_state->iter;  // (pipeline_begin synchronised the state)
  int64_t ahead = peer && c->x_ahead > 1 ? AHEAD_MAX : c->x_ahead, capf = c->x_fixed ? c->x_fixed : c->x_capf;
  // the last merge's record: the host's copy of the log range the last batch could write, pulled
  // with its poll (round 5 paid another host round trip per poll for it)
  int64_t lfrom = -1, ln = 0;
  bool pulled = false;  // (the run's merge records pulled by the last poll)
  auto last_rec = [&](LogRec* lr) -> int {
    const int64_t i = (int64_t)c->h_state->iter - 1;
    if (i >= lfrom && i < lfrom + ln) {
      *lr = c->x_hlog[i - lfrom];
    } else if (i == c->x_last_i) {  // (the previous run's last poll pulled it)
      *lr = c->x_last;
    } else {
      HIPCHK(c, hipMemcpy(lr, c->D.log + i, sizeof *lr, hipMemcpyDeviceToHost));
    }
    c->x_last = *lr;
    c->x_last_i = i;
    return 0;
  };
  while (!rc && done < n_merges) {
    // the middle regime once the winner's count is small (a poll is a quiescent point: the
    // lists are built, or rebuilt after an iteration stalled on them).  The decision and the
    // poll window read only replicated data -- the winner's global count from the replicated
    // counts, the iteration number -- so every rank switches at the same poll and issues the
    // same collectives (a rank's own merged count would let ranks part ways)
    // (the peer exchange stalls only past 2^19 records a rank: its batches run to the next
    // predicted switch, as the one-rank loop's do, instead of doubling from 1)
    int64_t win = ahead;
    const bool may_collapse = c->collapse_on && c->cg_ready && !c->ev && x_collapse_pays(c, n_merges - done);
    if ((!c->mid_on || may_collapse) && mid_enabled(c) && c->h_state->iter > 0) {
      LogRec lr;
      if ((rc = last_rec(&lr))) break;
      if (lr.count <= collapse_at && may_collapse) {
        // stop sharding: every rank takes the whole corpus and goes on alone (x_collapse)
        bool collapsed = false;
        if (peer) x_check_all(c);
        if ((rc = geobpe_pipeline_end(c)) || (rc = x_collapse(c, &collapsed))) return rc;
        if (collapsed) {
          int64_t more = 0;
          rc = geobpe_run(c, n_merges - done, &more);
          if (n_done) *n_done = done + more;
          return rc;
        }
        if ((rc = geobpe_pipeline_begin(c))) return rc;  // (some rank declined: sharded, as before)
      }
      if (!c->mid_on && lr.count <= mid_at) {
        c->mid_on = true;
        // the middle regime's records are per (workgroup, key), not per owner and key: a
        // merge of the same size sends up to ~4x as many -- a slot that small would stall
        if (!c->x_fixed) capf = std::min(CAP_MAX, 4 * capf);
      } else if ((!c->mid_on && lr.count <= 2 * mid_at) || (may_collapse && lr.count <= 2 * collapse_at)) {
        // (close to a switch: poll sooner -- at the predicted merge + 8 when the decay is known)
        const int64_t th = !c->mid_on && lr.count <= 2 * mid_at ? mid_at : collapse_at;
        int64_t w = 8;
        if (peer && c->x_decay > 0 && c->x_decay < 1 && lr.count > th)
          w = std::max<int64_t>(8, std::min<int64_t>(AHEAD_MAX, (int64_t)(std::log((double)th / lr.count) /
                                                                             std::log(c->x_decay)) + 8));
        win = std::min<int64_t>(win, w);
      }
    }
    if (c->mid_on && (rc = mid_prepare(c))) break;
    const int64_t slot = (1 + capf) * REC;
    const int64_t k = std::min(win, n_merges - done);  // an iteration merges at most once
    // the run's last batch (peer exchange): spec more iterations, idle on the device once the
    // batch's merges are made -- a hot-list rebuild iteration inside the batch then needs no
    // top-up batch and poll (run_batches' rule; the select's run_end)
    const int64_t extra = peer && k == n_merges - done ? c->spec : 0;
    const int32_t run_end = extra ? (int32_t)(c->h_state->iter + k + 1) : 0;
    for (int64_t i = 0; i < k + extra && !rc; i++) {
      if ((rc = pipeline_iter_impl(c, c->x_pbuf, c->x_pcap, peer, run_end))) break;
      if (peer) continue;  // (the records went to every peer inside the kernels; exchange.h)
      if ((rc = x_allgather(c, c->x_pbuf, c->x_gath, slot))) break;
      rc = geobpe_pipeline_import(c, c->x_gath, (int32_t)W, capf);
    }
    if (!rc && peer) rc = x_drain(c);  // (the batch's last records: the poll sees complete counts)
    const bool last = k == n_merges - done;  // (the run ends at this poll unless merges fell short)
    pulled = false;
    if (!rc && last) {  // (the end's work inside this poll's synchronisation: no second one)
      if (peer) x_check_all(c);
      if (log_first && !(rc = grow_h_log(c, it0 + n_merges + 1))) {
        flush_place(c);  // (the last place sums the last merge's merged occurrences into its record)
        const int64_t m = std::min<int64_t>(n_merges, c->h_log_cap - it0);
        if (m > 0) {
          const hipError_t e = hipMemcpyAsync(c->h_log + it0, c->D.log + it0, m * sizeof(LogRec),
                                              hipMemcpyDeviceToHost, c->stream);
          if (e != hipSuccess) rc = fail(c, GEOBPE_EHIP, "log pull: %s", hipGetErrorString(e));
        }
        pulled = true;
      }
    }
    if (!rc) {  // (the records the batch could write, pulled with the poll's synchronisation)
      lfrom = c->h_state->iter;
      ln = std::max<int64_t>(0, std::min<int64_t>({k, AHEAD_MAX + 2, c->D.KC - lfrom}));
      if (ln > 0) {
        const hipError_t e = hipMemcpyAsync(c->x_hlog, c->D.log + lfrom, ln * sizeof(LogRec), hipMemcpyDeviceToHost,
                                            c->stream);
        if (e != hipSuccess) rc = fail(c, GEOBPE_EHIP, "log pull: %s", hipGetErrorString(e));
      }
    }
    const double xt2 = xt ? now_us() : 0;
    if (rc || (rc = geobpe_pipeline_poll(c, out))) break;
    if (xt) fprintf(stderr, "xtime: batch of %lld enqueued at +%.1f us, poll %.1f us\n", (long long)k, xt2 - xt0,
                    now_us() - xt2);
    const bool stalled = out[0] != 0, fin = out[2] != 0;
    const int64_t it = out[1], smax = out[3];
    if (it - 1 >= lfrom && it - 1 < lfrom + ln) {  // (the next run's first decision needs no copy)
      c->x_last = c->x_hlog[it - 1 - lfrom];
      c->x_last_i = it - 1;
    }
    {  // the winner count's decay over the batch (the next batch's length near a switch)
      const int64_t z = std::min<int64_t>(it - 1, lfrom + ln - 1);
      if (ln > 0 && z > lfrom && c->x_hlog[0].count > 0 && c->x_hlog[z - lfrom].count > 0)
        c->x_decay = std::pow((double)c->x_hlog[z - lfrom].count / (double)c->x_hlog[0].count, 1.0 / (double)(z - lfrom));
    }
    if (stalled) {
      if ((rc = x_resolve(c))) break;
      ahead = 1;
    } else {
      ahead = peer ? AHEAD_MAX : std::min<int64_t>(2 * ahead, AHEAD_MAX);
    }
    if (!c->x_fixed) {
      int64_t p2 = 1;
      while (p2 < 2 * std::max<int64_t>(smax, 1)) p2 <<= 1;
      capf = std::min(CAP_MAX, std::max(CAP_MIN, p2));
    }
    done = it - it0;
    c->x_ahead = ahead;
    c->x_capf = capf;
    if (fin) break;
  }
  // (the last poll synchronised everything when the run ended with the batch it planned as its last)
  const bool fresh = pulled || (!log_first && c->enq == c->enq_synced && !c->place_pending);
  if (!rc && peer && !fresh) x_check_all(c);  // (the last imports' found keys: checked now, not by the next run)
  if (!rc && log_first && !pulled && !(rc = grow_h_log(c, it0 + n_merges + 1))) {
    // (the run's records in the end's own synchronisation; after the last place, which sums the
    // last merge's merged occurrences into its record)
    flush_place(c);
    const int64_t m = std::min<int64_t>(n_merges, c->h_log_cap - it0);
    if (m > 0) {
      const hipError_t e = hipMemcpyAsync(c->h_log + it0, c->D.log + it0, m * sizeof(LogRec), hipMemcpyDeviceToHost,
                                          c->stream);
      if (e != hipSuccess) rc = fail(c, GEOBPE_EHIP, "log pull: %s", hipGetErrorString(e));
    }
  }
  if (!rc && log_first) *log_first = it0;
  const int rc_end = fresh && !rc ? pipeline_end_lite(c) : geobpe_pipeline_end(c);
  if (rc) return rc;  // (an error in flight is the one to report)
  if (rc_end) return rc_end;
  if (n_done) *n_done = done;
  if (xt) fprintf(stderr, "xtime: run %.1f us\n", now_us() - xt0);
  return 0;
}

}  // namespace
