// exchange.h -- the peer exchange of the row-sharded loop (geobpe_comm_peer,
// geobpe_run_exchange).  Included once, by kernels.h, before merge.h and mid.h.
//
// Every rank holds the replicated global pair counts; after a merge each rank's count changes
// go to every other rank as 40-B delta records (content hash, length, representative, delta).
// Round 3-5 moved them with one ncclAllGather of fixed slots per merge plus an import kernel:
// two more stream operations and their gaps, ~30 us per heavy merge at world 1.  Here the
// records travel inside the kernels that make them:
//   producer (k_commit / k_mid_find, their exchange instantiations): record j of this rank is
//     stored into rank q's receive area at [parity][this rank] for every q != this rank
//     (x_put_rec, device.h) -- IPC-mapped device memory, xGMI stores on a node, write-through
//     (relaxed system-scope 8-B stores: nothing dirty left in an XCD's L2), no collective; the
//     rank's own deltas are applied at once by the producer.  Each workgroup waits for its stores
//     (s_waitcnt 0) and arrives on a counter; the last to arrive issues one system-scope release
//     and stores the slot header {count, seq} into every peer's area: x_arrive
//   wait: before the next select launch the host enqueues hipStreamWaitValue32 on the peer's
//     header seq (two ranks: the command processor waits) or one one-wave k_xwait kernel spinning
//     on every peer's (three or more: one launch instead of a stream wait per peer); bounded
//   import (the next select launch's place workgroups, before their place work): the other
//     ranks' records of that launch, found or claimed by content hash, added to the counts with
//     the hot-list check: x_import_share; the select workgroup waits for them (a counter of the
//     same launch) before its argmax.  A world-1 rehearsal (x_loop) stores its own records into
//     its own slot and imports them the same way
// A header count past the slot's capacity stalls every rank's pipeline (they all read the same
// headers); the host then re-exchanges that merge in full (x_resolve) and releases it.
#pragma once
// (included inside namespace gb)

struct XHdr {  // a receive slot's header (XHDR bytes)
  int64_t count;  // records of the source rank (-1: its launch did nothing, the pipeline stalled)
  int32_t seq;    // the producer launch's sequence number (the host's count of producer launches)
  int32_t pad;
};
static_assert(sizeof(XHdr) <= XHDR, "slot header");

__device__ inline XHdr* x_hdr(uint8_t* half, int64_t slot, int32_t src) {
  return reinterpret_cast<XHdr*>(half + (int64_t)src * slot);
}

// the end of a producer launch, every workgroup (block-uniform): its record stores made
// visible at system scope, then the arrival; the last workgroup publishes the slot headers
// (to every peer) and, for this rank's own import, the state
__device__ __attribute__((always_inline)) inline void x_arrive(const Dev& D) {
  if (D.xw == 0) return;
  // each wave's write-through stores into the peers' memory complete (vmcnt 0) -- no L2
  // write-back per wave: round 6's first form fenced every wave at system scope, a
  // buffer_wbl2 each, and the rehearsal's window fell from 8.8 k to 4.1 k merges/s
  if (D.xw > 1 || D.xloop) __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x != 0) return;
  State* st = D.st;
  const int32_t n = __hip_atomic_fetch_add(&st->xarr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (n != (int32_t)gridDim.x - 1) return;
  if (D.xw > 1 || D.xloop) __threadfence_system();  // (one release at system scope before the headers)
  st->xarr = 0;  // (the next producer launch comes after a kernel boundary)
  const bool stalled = __hip_atomic_load(&st->stall, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  const int64_t cnt =
      stalled ? -1 : (int64_t)__hip_atomic_load((unsigned long long*)D.xcnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int q = 0; q < XPEER_MAX; q++) {  // (static indices into D.xpeer: see x_put_rec)
    if (q >= D.xw || (q == D.xme && !D.xloop)) continue;
    XHdr* h = x_hdr(D.xpeer[q], D.xslot, D.xme);
    __hip_atomic_store(&h->count, cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&h->seq, D.xseq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (!stalled) {  // (a stalled pipeline keeps the stalled merge's state for the full re-exchange)
    st->xpcnt = cnt;
    st->xppar = D.xpar;
    st->xpseq = D.xseq;
    st->xpend = 1;
  }
}

// What the import workgroups write that the select workgroup of the same launch reads (the
// hot-list entries, a claimed key's content) is written through to memory (agent-scope relaxed
// atomic stores: no dirty line in an XCD's L2); the counts are atomics.  So an import workgroup
// ends with its stores complete (vmcnt 0) and a relaxed arrival, and the select workgroup with
// one acquire (its L2 invalidated) -- a release / acquire pair per workgroup is an L2 write-back
// and invalidate per workgroup, and 32 of them per XCD cost the first form ~60 us a launch.
__device__ inline void x_hot_store(const Dev& D, int64_t k, int32_t d) {
  if (k < D.KCAP)
    __hip_atomic_store(&D.clist[k], d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    __hip_atomic_store(&D.st->cl_valid, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void x_count_add_hot(const Dev& D, HotApp& h, int32_t d, int32_t v, int32_t th) {
  const int32_t old = atomicAdd(&D.count[d], v);
  if (v > 0 && th > 0 && old < th && old + v >= th) {
    const int32_t j = atomicAdd(&h.n, 1);
    if (j < HOT_BUF)
      h.buf[j] = d;
    else
      x_hot_store(D, (int64_t)atomicAdd((unsigned long long*)&D.st->ncl2[D.st->cl_act], 1ULL), d);
  }
}
__device__ inline void x_hot_flush(const Dev& D, HotApp& h) {
  __shared__ int64_t s_base;
  __syncthreads();
  const int32_t n = min(h.n, HOT_BUF);
  if (threadIdx.x == 0 && n > 0)
    s_base = (int64_t)atomicAdd((unsigned long long*)&D.st->ncl2[D.st->cl_act], (unsigned long long)n);
  __syncthreads();
  for (int32_t i = threadIdx.x; i < n; i += blockDim.x) x_hot_store(D, s_base + i, h.buf[i]);
}
__device__ inline void x_claim_payload(const Dev& D, int32_t slot, const DeltaRec& r) {
  __hip_atomic_store((unsigned long long*)&D.kh1[slot], (unsigned long long)r.h1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store((unsigned long long*)&D.kh2[slot], (unsigned long long)r.h2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&D.klen[slot], r.len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&D.krep[3 * (int64_t)slot], r.idL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&D.krep[3 * (int64_t)slot + 1], r.g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&D.krep[3 * (int64_t)slot + 2], r.idR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct XImpLds {
  HotApp hot;
  int64_t pre[XPEER_MAX + 1];  // record prefix over the ranks
  int32_t ns, go, bad, chk, half;
};

// a claimed key of import workgroup b joins klist at the end (region b of D.ns)
__device__ inline void x_note_claim(const Dev& D, XImpLds& X, int32_t b, int32_t slot) {
  const int32_t j = atomicAdd(&X.ns, 1);
  if (j < D.RC)
    D.ns[(int64_t)b * D.RC + j] = slot;
  else
    klist_put(D, (int64_t)atomicAdd((unsigned long long*)&D.st->U, 1ULL), slot);
}

// a key the import found (not claimed) is checked against its stored content by the next import
// of the same workgroup index: another import workgroup of this launch may have claimed it and
// not yet written the content (the deferred check of k_import_fixed's emit_check).  The regions
// come in two halves by the import's producer sequence number (h = seq & 1): an import writes
// half h and, after its arrival -- off the select's path -- checks half h ^ 1, the last import's
// (round 6's first form checked first: three dependent rounds before every import's own loads)
__device__ inline int64_t x_chk_region(const Dev& D, int32_t h, int32_t b) { return (int64_t)h * D.NBA + b; }
__device__ inline void x_note_found(const Dev& D, XImpLds& X, int32_t b, int32_t d, const DeltaRec& r) {
  const int32_t j = atomicAdd(&X.chk, 1);
  if (j < D.xchkcap) {
    NewPair e;
    e.target = d;
    e.slot = -1;
    e.len = r.len;
    e.delta = 0;
    e.h1 = r.h1;
    e.h2 = r.h2;
    D.xchk[x_chk_region(D, X.half, b) * D.xchkcap + j] = e;
  } else {
    atomicAdd((unsigned long long*)&D.st->nunchecked, 1ULL);
  }
}
// an import's found keys (region r = x_chk_region), against the key table (EHASH); the region is
// then empty (block-uniform)
__device__ inline void x_check_region(const Dev& D, int64_t r) {
  const int32_t n = min(D.xchkcnt[r], (int32_t)D.xchkcap);
  for (int32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const NewPair e = D.xchk[r * D.xchkcap + i];
    if (!key_is(D, e.target, e.h1, e.h2, e.len)) set_error(D, GEOBPE_EHASH, -81);
  }
  __syncthreads();  // (every thread has read the count)
  if (threadIdx.x == 0 && n > 0) D.xchkcnt[r] = 0;
}

// a relaxed system-scope load (a record another device stored: not through a stale L2 line)
__device__ inline DeltaRec x_load_rec(const DeltaRec* p) {
  DeltaRec r;
  const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
  unsigned long long* o = reinterpret_cast<unsigned long long*>(&r);
#pragma unroll
  for (int i = 0; i < 5; i++) o[i] = __hip_atomic_load(q + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return r;
}

// the import's end: the counters the producer used start again (the stalled case keeps this
// rank's record count and the pending flag for the host's full re-exchange)
__device__ inline void x_import_finish(const Dev& D) {
  State* st = D.st;
  st->xiarr = 0;
  st->ntouched = 0;
  st->nxovf = 0;  // (k_commit turned k_find's side list into records)
  st->epoch += 1;
  if (!st->stall) {
    *D.xcnt = 0;
    st->xpend = 0;
  }
  __threadfence();
}

// share b of nb of the pending records (block-uniform; every workgroup of the launch that
// takes a share calls it).  last_finishes: the last workgroup to arrive ends the import (the
// drain launch); else the select workgroup does, after waiting for all of them (x_import_wait).
__device__ void x_import_share(const Dev& D, XImpLds& X, int32_t b, int32_t nb, bool last_finishes) {
  State* st = D.st;
  const int32_t t = threadIdx.x;
  if (t == 0) {
    X.go = D.xw > 0 && st->xpend != 0;  // (stable for the whole launch: only the finish clears it)
    X.bad = st->stall != 0;
    X.half = st->xpseq & 1;
    X.ns = 0;
    X.chk = 0;
  }
  hot_init(X.hot);
  __syncthreads();
  if (!X.go) {  // (no import: both halves' found keys checked now -- their claims are complete)
    if (D.xw > 0) {
      x_check_region(D, x_chk_region(D, 0, b));
      x_check_region(D, x_chk_region(D, 1, b));
    }
    return;
  }
  const int32_t W = D.xw, par = st->xppar, seq = st->xpseq;
  uint8_t* half = D.xrecv + (int64_t)par * W * D.xslot;
  if (t < W && !X.bad) {  // every other rank's count from its header, one thread a rank (stalled:
                          // later no-op launches have overwritten them -- not read).  This rank's
                          // own records were applied by the producer (x_put_rec): none to import,
                          // but a count past the slots stalls every rank, this one included
    int64_t c = st->xpcnt > D.xcapf ? -1 : 0;
    if (t != D.xme || D.xloop) {
      XHdr* h = x_hdr(half, D.xslot, t);
      const int32_t sq = __hip_atomic_load(&h->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      c = __hip_atomic_load(&h->count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (sq != seq) {  // (the stream waited for it: a header of another launch is a protocol error)
        set_error(D, GEOBPE_ESTATE, -80);
        c = -1;
      }
    }
    X.pre[t + 1] = c;
  }
  __syncthreads();
  if (t == 0 && !X.bad) {
    int64_t acc = 0;
    X.pre[0] = 0;
    for (int q = 0; q < W; q++) {
      const int64_t c = X.pre[q + 1];
      if (c < 0 || c > D.xcapf) X.bad = 1;
      acc += max(c, (int64_t)0);
      X.pre[q + 1] = acc;
    }
    if (X.bad) st->stall = 1;  // (every rank reads the same headers: every rank stalls here)
  }
  __syncthreads();
  if (!X.bad) {
    const int32_t th = st->theta;
    const int64_t n = X.pre[W];
    const int64_t E = (n + nb - 1) / nb;
    const int64_t lo = (int64_t)b * E, hi = min(n, lo + E);
    for (int64_t j = lo + t; j < hi; j += ABLOCK) {
      int r = 0;
      while (j >= X.pre[r + 1]) r++;
      const int64_t k = j - X.pre[r];
      const DeltaRec rr = x_load_rec(reinterpret_cast<const DeltaRec*>(half + (int64_t)r * D.xslot + XHDR) + k);
      if (rr.delta == 0) continue;
      bool claimed;
      const int32_t d = ht_insert(D, rr.h1, rr.h2, rr.len, &claimed);
      if (d < 0) continue;
      if (claimed) {
        x_claim_payload(D, d, rr);
        x_note_claim(D, X, b, d);
      } else {
        x_note_found(D, X, b, d, rr);
      }
      x_count_add_hot(D, X.hot, d, rr.delta, th);
    }
  }
  x_hot_flush(D, X.hot);  // (syncs the workgroup first)
  {  // this workgroup's claims join klist
    __shared__ int64_t s_base;
    __syncthreads();
    const int32_t m = min(X.ns, (int32_t)D.RC);
    if (t == 0) s_base = m ? (int64_t)atomicAdd((unsigned long long*)&st->U, (unsigned long long)m) : 0;
    __syncthreads();
    for (int32_t i = t; i < m; i += ABLOCK) klist_put(D, s_base + i, D.ns[(int64_t)b * D.RC + i]);
  }
  if (t == 0) D.xchkcnt[x_chk_region(D, X.half, b)] = min(X.chk, (int32_t)D.xchkcap);
  __builtin_amdgcn_s_waitcnt(0);  // (this wave's stores and atomics complete)
  __syncthreads();
  if (t == 0) {
    const int32_t a = __hip_atomic_fetch_add(&st->xiarr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (last_finishes && a == nb - 1) x_import_finish(D);
  }
  // the last import's found keys (the other half): their claims are complete since that launch
  // ended -- checked after the arrival, while the select works
  x_check_region(D, x_chk_region(D, X.half ^ 1, b));
}

// the select workgroup: wait for the nb import workgroups of its launch (bounded: a protocol
// error, not a hang), then end the import.  Returns false when the pipeline is stalled.
__device__ inline bool x_import_wait(const Dev& D, bool pending, int32_t nb) {
  State* st = D.st;
  __shared__ int32_t s_ok;
  if (threadIdx.x == 0) {
    s_ok = 1;
    if (pending) {
      const uint64_t t0 = wall_clock64();
      // (relaxed loads in the loop, one acquire after it: an acquire load per iteration is an
      // L2 invalidate per iteration, under the import and place workgroups of this launch)
      while (__hip_atomic_load(&st->xiarr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < nb) {
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() - t0 > (uint64_t)100000000) {  // (~1 s at the 100 MHz wall clock)
          set_error(D, GEOBPE_ESTATE, -82);
          st->stall = 1;
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      x_import_finish(D);
    }
    s_ok = __hip_atomic_load(&st->stall, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
  }
  __syncthreads();
  return s_ok != 0;
}

// the end of a peer-exchange run: every import region's found keys checked (the imports of the
// next run would check them otherwise)
__global__ __launch_bounds__(ABLOCK) void k_xcheck(Dev D) {
  x_check_region(D, x_chk_region(D, 0, blockIdx.x));
  x_check_region(D, x_chk_region(D, 1, blockIdx.x));
}

// the drain at the end of a batch: the last producer launch's records, imported on their own
__global__ __launch_bounds__(ABLOCK) void k_xdrain(Dev D) {
  __shared__ XImpLds X;
  x_import_share(D, X, blockIdx.x, gridDim.x, true);
}
