/*
 * geobpe.h -- C-ABI of the MI355X-native GeoBPE merge loop (libgeobpe.so).
 *
 * The reference has no FFI: its hot path is the Python object API of
 * foldingdiff.bpe.BPE.  Each entry point below replaces one
 * step of that API; the Python host mirror (pt-bpe_amd/geobpe/bpe.py) binds them
 * with ctypes exactly where the reference calls the Python methods.
 *
 * Conventions: plain pointers and sizes, no torch types.  Host pointers are
 * marked h_, device pointers d_.  Every call is ordered on the context's HIP
 * stream (the stream given at create time, or a private one).  Every function
 * returns 0 on success and a nonzero GEOBPE_E* code on failure; the message is
 * in geobpe_last_error().  GEOBPE_EVALUE corresponds to the reference's
 * ValueError from BPE.get_ind (foldingdiff/bpe.py:1180-1189).
 */
#ifndef GEOBPE_H
#define GEOBPE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GEOBPE_OK 0
#define GEOBPE_EARG 1      /* bad argument / call order */
#define GEOBPE_EVALUE 2    /* a value outside the histogram range (reference ValueError) */
#define GEOBPE_ECAPACITY 3 /* a device table is full */
#define GEOBPE_EHIP 4      /* HIP runtime error */
#define GEOBPE_EHASH 5     /* content-hash collision detected (never expected) */
#define GEOBPE_ESTATE 6    /* inconsistent device token links (internal error; never expected) */

/* angle column order of the input table (= Tokenizer.init_structure,
 * foldingdiff/tokenizer.py:393-405): */
#define GEOBPE_COL_0C1N 0
#define GEOBPE_COL_NCA 1
#define GEOBPE_COL_CAC 2
#define GEOBPE_COL_PHI 3
#define GEOBPE_COL_PSI 4
#define GEOBPE_COL_OMEGA 5
#define GEOBPE_COL_TAU 6
#define GEOBPE_COL_CAC1N 7
#define GEOBPE_COL_C1NCA 8
/* threshold type order (= BPE._init_thresholds keys, bpe.py:828):
 * tau, CA:C:1N, C:1N:1CA, psi, omega, phi */
#define GEOBPE_NTYPES 6

typedef struct geobpe_ctx geobpe_ctx;

/* Create a context on HIP device `device`.  `stream` is a hipStream_t (e.g.
 * torch.cuda.current_stream().cuda_stream) or NULL for a private stream.
 * `max_vocab` bounds len(_tokens) (K0 + merges). */
int geobpe_create(geobpe_ctx **out, int device, void *stream, int64_t max_vocab);
void geobpe_destroy(geobpe_ctx *ctx);
const char *geobpe_last_error(geobpe_ctx *ctx);

/* ---- prologue: BPE.__init__ + BPE.initialize() (bpe.py:33-103, 820-876, 138-394) ----
 * Upload the corpus: n_rows chains, h_row_off[n_rows+1] residue offsets and the
 * 9 float64 columns (each h_cols[c] has row_off[n_rows] values, NaN allowed). */
int geobpe_load_angles(geobpe_ctx *ctx, int64_t n_rows, const int64_t *h_row_off, const double *const *h_cols);

/* Per threshold type t (order above): min and max of the wrapped, non-NaN,
 * non-zero column values (bpe.py:844 + plotting.py:309-310), and how many
 * there were.  h_minmax[2t] = min, [2t+1] = max; h_count[t].  The tau init
 * angle of bpe.py:845-846 is NOT included (the host adds it). */
int geobpe_angle_range(geobpe_ctx *ctx, double *h_minmax, int64_t *h_count);

/* Set the grid-1 histogram edges (np.histogram edges, B+1 per type, type-major)
 * and quantise every residue / junction (get_ind semantics, bpe.py:1164-1189).
 * `init_tau` is Tokenizer._init_bond_angle (tokenizer.py:74-77).
 * Fails with GEOBPE_EVALUE if any used value falls outside its bins. */
int geobpe_quantize(geobpe_ctx *ctx, int32_t B, const double *h_edges, double init_tau);

/* First appearance of every residue symbol: h_first[s] = smallest residue index
 * (+ row_base) holding symbol s, or INT64_MAX.  Symbols s < B^3 + B. */
int geobpe_symbol_first(geobpe_ctx *ctx, int64_t row_base, int64_t *h_first);

/* Install the initial residue tokens: label of symbol s = h_label_of_sym[s]
 * (first-appearance rank, bpe.py:231-261); K0 labels. */
int geobpe_init_tokens(geobpe_ctx *ctx, const int32_t *h_label_of_sym, int32_t K0);

/* ---- BPE.bin(): full content-keyed adjacent-pair histogram (bpe.py:1431-1474) ---- */
int geobpe_bin(geobpe_ctx *ctx);
/* Bin-pass form: 1 (default) = dense symbol-triple histogram when the corpus
 * is at its initial state and K0*B^3*K0 <= 2^26; 0 = per-pair key probing.
 * Both produce the same keys, counts and pk; must precede geobpe_bin(). */
int geobpe_set_bin_dense(geobpe_ctx *ctx, int on);

/* ---- BPE.step() (bpe.py:1792-2166) ----
 * One merge iteration: device argmax (max count, ties -> smallest reference key
 * string: SortedDict.peekitem(0), bpe.py:1796-1800), greedy non-overlapping
 * merge-apply (bpe.py:1888-2014), incremental count update, new token
 * _tokens[n] = json.loads(key) (bpe.py:1857-1860).
 * *new_id = the new token id (len(_tokens) before the step), *count = its
 * occurrence count, *n_merged = merges applied; *new_id = -1 if no pair is left. */
int geobpe_step(geobpe_ctx *ctx, int32_t *new_id, int32_t *count, int64_t *n_merged);

/* Enqueue n_iters merge iterations back to back with no host synchronisation
 * (the winner, tie-break and new token are resolved on the device), then wait;
 * *n_done = merges actually made (fewer if the pairs ran out). */
int geobpe_run(geobpe_ctx *ctx, int64_t n_iters, int64_t *n_done);
/* geobpe_run, and the merges it made in h_out (3 int64 per merge, as geobpe_merge_log;
 * at most cap); *first = the merges made before this run.  Their log records ride in the
 * run's own state synchronisations to a pinned mirror, so the caller's merge list needs no
 * further round trip (BPE.step's per-step bookkeeping of the merge list,
 * bpe.py:1857-1866).  Single rank. */
int geobpe_run_log(geobpe_ctx *ctx, int64_t n_iters, int64_t *n_done, int64_t *first, int64_t *h_out,
                   int64_t cap);
/* Late-merge path (same results): once a merge's count is <= max_count, geobpe_run /
 * geobpe_step run the merges in one workgroup over per-key posting lists (k_tail, many
 * merges per launch) instead of the full-grid kernels; 0 = never (the default: the middle regime is faster;
 * environment GEOBPE_TAIL overrides at create).  Single rank, no merge replay. */
int geobpe_set_tail(geobpe_ctx *ctx, int64_t max_count);
/* Middle regime (same results): once a merge's count is <= max_count, merges run as two
 * launches (select + the previous merge's place, then find) over the per-key posting lists
 * (0 = never; default 49152; environment GEOBPE_MID overrides at create).  Single rank. */
int geobpe_set_mid(geobpe_ctx *ctx, int64_t max_count);
/* The merge list so far: 3 int64 per merge (new id, count, merges applied);
 * returns the number of merges (copies at most cap). */
int64_t geobpe_merge_log(geobpe_ctx *ctx, int64_t *h_out, int64_t cap);

/* The split step for row-sharded multi-GPU runs: select (argmax over the
 * replicated global counts) + apply locally, recording count deltas; then the
 * caller exchanges the delta records (geobpe_delta_export / _import). */
int geobpe_step_select(geobpe_ctx *ctx, int32_t *new_id, int32_t *count);
int geobpe_step_apply(geobpe_ctx *ctx, int64_t *n_merged);
/* Delta records (40 bytes each) of every key whose local count changed since
 * the last export; copies them to d_out (device, capacity cap records). */
int geobpe_delta_export(geobpe_ctx *ctx, void *d_out, int64_t cap, int64_t *n_records);
/* Add the records (from every rank, this one included) to the global counts. */
int geobpe_delta_import(geobpe_ctx *ctx, const void *d_in, int64_t n_records);
/* Stream-ordered variants (no host synchronisation): the export writes its
 * record count to d_count (device int64; GEOBPE_ECAPACITY at the next sync if it
 * exceeds cap); the import of n_records is only enqueued. */
int geobpe_delta_export_async(geobpe_ctx *ctx, void *d_out, int64_t cap, void *d_count);
int geobpe_delta_import_async(geobpe_ctx *ctx, const void *d_in, int64_t n_records);
/* 1 = multi-rank mode (local changes go to the delta buffer), 0 = single.
 * Must precede geobpe_bin(). */
int geobpe_set_distributed(geobpe_ctx *ctx, int on);
/* Pipelined multi-rank loop (no host wait per merge).  The
   reference has no distributed step (BPE.step, bpe.py:1792-2166, is serial); this
   replaces a host-synchronised step_select / step_apply / delta exchange per merge.
   Per iteration: geobpe_pipeline_iter enqueues select (+ the previous merge's place) /
   find / commit, which write this rank's delta records straight into
   d_buf = [header record: int64 count][records ... cap_total], and the header; the caller
   all-gathers the first (1 + cap_fixed) records of every rank's d_buf; then
   geobpe_pipeline_import consumes the gathered slots.  A rank whose count exceeds
   cap_fixed stalls every pipelined kernel; geobpe_pipeline_poll reports
   {stalled, merges, done, largest slot count of the last import} (the same on every
   rank: it sizes the next slots); after a stall the caller gathers the full records
   of that merge and calls geobpe_pipeline_resolve. */
int geobpe_pipeline_begin(geobpe_ctx *ctx);
int geobpe_pipeline_iter(geobpe_ctx *ctx, void *d_buf, int64_t cap_total);
int geobpe_pipeline_import(geobpe_ctx *ctx, const void *d_slots, int32_t world, int64_t cap_fixed);
int geobpe_pipeline_poll(geobpe_ctx *ctx, int64_t *h_out4);
int geobpe_pipeline_resolve(geobpe_ctx *ctx, const void *d_in, int64_t n_records);
int geobpe_pipeline_end(geobpe_ctx *ctx);
/* Residues of the whole (all-rank) corpus: sizes the replicated key table. */
int geobpe_set_global_residues(geobpe_ctx *ctx, int64_t n);
/* This context's rank in the exchange (pipelined import: its own slot's records carry
   their local key ids, so they are not probed again). */
int geobpe_set_rank(geobpe_ctx *ctx, int32_t rank);

/* ---- introspection / exports ---- */
/* Key string (json.dumps(geo, sort_keys=True)) of vocab id v's content. */
int64_t geobpe_token_json(geobpe_ctx *ctx, int32_t v, char *buf, int64_t cap);
/* Key string of pair key d (key id = key-table slot; introspection / tests). */
int64_t geobpe_key_json(geobpe_ctx *ctx, int32_t d, char *buf, int64_t cap);
/* Device ordering of reference key strings: h_out[i] = key(h_pairs[2i]) <
 * key(h_pairs[2i+1]) for key ids (tests the device tie-break of the
 * SortedDict order, bpe.py:1469-1471). */
int geobpe_debug_key_less(geobpe_ctx *ctx, const int32_t *h_pairs, int32_t n, int32_t *h_out);
/* Every klist entry (key id = key-table slot, in claim order; -1 = an unused
 * chunk entry) and its global pair count; returns the number of entries,
 * copies at most cap of each. */
int64_t geobpe_debug_counts(geobpe_ctx *ctx, int32_t *h_keys, int32_t *h_counts, int64_t cap);
/* debug: argmax state after a sync -- {hot-list length, theta, tied keys of the last
   merge, its count, rebuild iterations, list valid, merges, vocab, posting index valid,
   posting log length}; returns 10 (cap >= 10) */
int64_t geobpe_debug_state(geobpe_ctx *ctx, int64_t *h_out, int64_t cap);
/* Debug record of key d: idL, g, idR, len, count, U, K(device), K(host), h1. */
int geobpe_debug_key(geobpe_ctx *ctx, int32_t d, int64_t *h_out9);
/* Content (residue / junction symbols, 2*nres-1 values) of vocab id v. */
int64_t geobpe_token_content(geobpe_ctx *ctx, int32_t v, int32_t *h_out, int64_t cap);
int64_t geobpe_vocab_count(geobpe_ctx *ctx); /* len(_tokens) */
int64_t geobpe_num_keys(geobpe_ctx *ctx);    /* distinct pair keys ever seen (len of the reference's _geo_dict history) */
int64_t geobpe_num_tokens(geobpe_ctx *ctx);  /* live tokens (sync) */
/* Segmentation (Tokenizer.bond_to_token order, tokenizer.py:24-61): per row the
 * (start residue within the row, token id) of every token.  Call with NULL buffers to get the total count. */
int64_t geobpe_segmentation(geobpe_ctx *ctx, int32_t *h_start, int32_t *h_id, int64_t *h_row_tok_off);
/* quantize(tokenize()) of every row (tokenizer.py:379-392, bpe.py:918-956). */
int64_t geobpe_encode(geobpe_ctx *ctx, int32_t *h_ids, int64_t *h_row_id_off);
/* Full recount of the live pair histogram from the per-token key ids, compared
 * with the incrementally maintained counts: returns the number of mismatching
 * keys (0 = consistent), or -1 on error. */
int64_t geobpe_verify_counts(geobpe_ctx *ctx);
/* Per-kernel time (ms summed over launches, HIP events on the context stream)
 * while profiling is enabled.  names: "pair_count", "finalize", "bin_pack" (bin),
 * "select" (+ the previous merge's place), "find", "commit", "place" (a place
 * launched on its own), "recount".  The merge loop's k_commit also counts its work
 * (key / decrement records, keys: geobpe_debug_state) when on = 1.  on = 0: off; on = 1: every
 * launch; on = k > 1: every k-th launch of each kernel, from launch k / 2 (a run's first
 * launch starts cold).  The merge loop's single-kernel launches carry their events on their
 * own dispatch (hipExtLaunchKernelGGL: kernel start / end, no marker packets). */
int geobpe_set_profiling(geobpe_ctx *ctx, int on);
/* k_commit's work counters (key records, decrement records, keys: geobpe_debug_state
 * slots 10-12) on or off; geobpe_set_profiling with stride 1 turns them on (they slow
 * k_commit: a timing run turns them off after it). */
int geobpe_set_work_counters(geobpe_ctx *ctx, int on);
/* Timing aid: geobpe_run enqueues a kernel that spins for `us` microseconds before each
 * batch of iterations, so per-launch events measure kernels queued behind it rather than
 * the host's enqueue pace (0 = off, the default). */
int geobpe_set_hold(geobpe_ctx *ctx, int64_t us);
/* Debug: per-workgroup phase timestamps (wall clock, 100 MHz) of k_select / k_find /
 * k_commit / k_place (tools/debug/merge_timeline.py).
 * on = 1 enables and clears (returns the slot count); on = 0 copies up to cap
 * stamps to h_out and disables. */
int64_t geobpe_debug_timeline(geobpe_ctx *ctx, int on, int64_t *h_out, int64_t cap);
/* Restrict the timing to a comma-separated list of kernel names ("" = all). */
int geobpe_set_profiling_filter(geobpe_ctx *ctx, const char *names);
double geobpe_kernel_ms(geobpe_ctx *ctx, const char *name, int64_t *launches);
/* Profiling: enqueue k_window_mark (one empty workgroup) on the engine stream.
 * bench.py brackets its timed region with two of them (outside the timer) so a
 * rocprofv3 trace / PMC pass can select exactly that window's dispatches. */
int geobpe_marker(geobpe_ctx *ctx, int32_t tag);
/* ---- PDB -> internal coordinates (the reference's
 * canonical_distances_and_dihedrals, foldingdiff/angles_and_coords.py:69-154) ----
 * geobpe_pdb_backbone: N, CA, C (x, y, z) of every amino-acid residue of the
 * first model, 9 doubles per residue; returns the residues (h_xyz NULL: count
 * only) or -GEOBPE_E* (-GEOBPE_EVALUE: a residue lacks a backbone atom, the
 * reference's BadStructureError); geobpe_pdb_error() has the message.
 * geobpe_featurize: on the device, the nine columns (GEOBPE_COL_* order, R values
 * each) of chains given by row_off[n_rows+1] over the residues of h_xyz. */
int64_t geobpe_pdb_backbone(const char *path, double *h_xyz, int64_t cap_residues);
const char *geobpe_pdb_error(void);
int geobpe_featurize(int device, int64_t n_rows, const int64_t *h_row_off, const double *h_xyz,
                     double *const *h_cols);

/* ---- merge replay (bin/induce.py: encode new chains with a trained vocabulary;
 * SURVEY.md §8(f) row 1) ----
 * After bin() and before any merge: merge t of geobpe_run / geobpe_step becomes
 * the trained token K0 + t -- content hash (h1, h2) of len residues and one split
 * L ++ [g] ++ R into earlier token ids -- instead of the argmax.  Every occurrence
 * is merged greedily left to right as in training; a content with no occurrence
 * merges nothing but keeps its token id.  geobpe_run stops after n merges (done).
 * The context must have been initialised with the trained grid and labels
 * (geobpe_quantize edges, geobpe_init_tokens label map). */
int geobpe_replay_load(geobpe_ctx *ctx, const uint64_t *h_h1, const uint64_t *h_h2, const int32_t *h_len,
                       const int32_t *h_idL, const int32_t *h_g, const int32_t *h_idR, int64_t n);

/* ---- merge events: the checkpoint's merge tree (TokenHierarchy.__setitem__ ->
 * BinaryTreeBuilder.combine, data_structures.py:32-60,217-226) ----
 * on=1 before the first merge: every merged occurrence of every later merge is
 * logged on the device.  geobpe_events copies (merge index, left token start
 * slot, right token start slot) of all logged events (any order within a merge)
 * and returns their number (-1: not recording / error); NULL buffers: count only. */
/* Kabsch RMSD of structure pairs (no context needed).
   h_a: n_a structures x n_atoms x 3 float64; h_b likewise (ignored when symmetric);
   h_out[i * n_b + j] = compute_rmsd(A_i, B_j) of foldingdiff/algo.py:48-65 (Q = B_j
   aligned onto P = A_i by kabsch, algo.py:8-46).  symmetric: B = A, the upper
   triangle is computed and mirrored (k_medoids' distance matrix, algo.py:179-189).
   Replaces the joblib-threaded compute_rmsd loops of k_medoids and the medoid
   assignment (bpe.py:645-657, 1764-1777). */
int geobpe_rmsd(int device, int32_t n_a, int32_t n_b, int32_t n_atoms, const double *h_a, const double *h_b,
                int symmetric, double *h_out);
/* NeRF: token coordinates from internal coordinates (Tokenizer.geo_nerf,
   tokenizer.py:317-344, NERFBuilder / place_dihedral, nerf.py:85-211, the first
   residue by update_backbone_positions, angles_and_coords.py:238-316), one span of
   whole residues per thread.  h_res_off[n_spans + 1]: residue offsets; h_geo: 9
   float64 per residue {N:CA, CA:C, tau, 0C:1N, CA:C:1N, C:1N:1CA, psi, omega, phi}
   (the last six: the junction to the next residue of the span); h_xyz: N, CA, C of
   every residue (9 float64 per residue). */
int geobpe_nerf(int device, int64_t n_spans, const int64_t *h_res_off, const double *h_geo, double *h_xyz);
/* Glue optimisation of the RMSD mode: L-BFGS (torch.optim.LBFGS, max_iter 20,
   strong-Wolfe line search) over every glue triple (omega_k, C:1N:1CA_k, phi_k) of each
   chain, minimising the exit-frame loss of the chain's NeRF against cached frames plus the
   optional von Mises prior.  Replaces BPE.glue_opt_all / _opt_glue_worker / opt_glue /
   optimize_glues_entry_torch / fk_segment_torch (bpe.py:106-135, 423-578, 739-807), one
   64-lane wave per chain (k_glue_wave: prefix-product NeRF, suffix-sum gradient; environment
   GEOBPE_GLUE_THREAD=1 selects the one-thread-per-chain k_glue_opt).  h_res_off[n_chains + 1]: residue offsets; h_geo: 9 float64 per
   residue (geobpe_nerf's layout, float32-representable values); per glue (r - 1 per
   chain, in order): h_x0 3 float32 (raw start values), h_tgt 12 float32 (target frame R
   row-major, then t); h_grid[n_chains]: prior table per chain; h_prior: n_grid x 3 types
   (omega, C:1N:1CA, phi) x {centres[kmax], weights[kmax]}; h_kcnt: n_grid x 3 bin
   counts; lam: glue_opt_prior; w_rot / w_trans: wR / wt.  Out: h_xout 3 float32 per glue
   (the wrapped optimum, before snapping), h_stats 2 per chain (iterations, evaluations),
   h_loss 2 per chain (first and last loss). */
int geobpe_glue_opt(int device, int64_t n_chains, const int64_t *h_res_off, const double *h_geo, const float *h_x0,
                    const float *h_tgt, const int32_t *h_grid, int32_t n_grid, int32_t kmax, const float *h_prior,
                    const int32_t *h_kcnt, float lam, double w_rot, double w_trans, float *h_xout, int32_t *h_stats,
                    double *h_loss);
/* The context-free entry points above (geobpe_rmsd / geobpe_nerf / geobpe_glue_opt) keep one
   stream and one grown scratch arena per (device, entry point), each behind its own lock.
   This frees the arenas of `device` (-1: every device); the next call re-creates them. */
int geobpe_arena_release(int device);
int geobpe_set_record_events(geobpe_ctx *ctx, int on);
int64_t geobpe_events(geobpe_ctx *ctx, int32_t *h_merge, int32_t *h_a, int32_t *h_b);

int geobpe_synchronize(geobpe_ctx *ctx);

/* ---- the engine's own multi-rank exchange (replaces the host-driven collectives of
 * geobpe/dist.py TorchGroup.run_pipelined; the reference has no multi-GPU path) ----
 * An RCCL communicator owned by the engine: rank 0 makes the 128-byte id, the caller
 * broadcasts it, every rank attaches.  rccl_path: the RCCL library the process already
 * uses (PyTorch's), NULL = "librccl.so.1". */
int geobpe_comm_unique_id(const char *rccl_path, void *out128);
int geobpe_comm_init_rccl(geobpe_ctx *ctx, const char *rccl_path, const void *unique_id, int32_t nranks,
                          int32_t rank);
const char *geobpe_comm_error(void);
/* Or a host collective: fn gathers `bytes` host bytes from every rank, rank-major, into
 * recv (nranks * bytes); called synchronously by geobpe_run_exchange (tests over gloo). */
typedef int (*geobpe_allgather_fn)(void *user, const void *send, void *recv, int64_t bytes);
int geobpe_comm_set_callback(geobpe_ctx *ctx, geobpe_allgather_fn fn, void *user, int32_t nranks, int32_t rank);
/* Fixed slot size in records (0 = sized from the last import; tests force stalls with it). */
int geobpe_comm_set_slot(geobpe_ctx *ctx, int64_t records);
/* The peer exchange (default on for up to 8 ranks; off: the all-gather of fixed slots): every
 * rank's receive area is IPC-mapped into every other rank once, the merge kernels store their
 * delta records straight into the peers' areas and publish a {count, seq} header, the stream
 * waits for the peers' headers (hipStreamWaitValue32 with two ranks, a one-wave waiter kernel with
 * more; bounded) and the next select launch imports them.
 * GEOBPE_PEER=0 in the environment turns it off too.  Set before the first geobpe_run_exchange.
 * (No reference counterpart: the reference has no multi-GPU path) */
int geobpe_comm_peer(geobpe_ctx *ctx, int on);
/* 1 when geobpe_run_exchange runs the peer exchange (set up and agreed on by every rank). */
int geobpe_comm_peer_active(geobpe_ctx *ctx);
/* At the middle-regime switch (the winner's global count <= geobpe_set_mid's threshold),
 * geobpe_run_exchange stops sharding: every rank gathers every rank's token records once,
 * re-keys them in its own key table and continues as the one-rank loop over the whole corpus
 * (no exchange per merge; every rank makes the same merges).  Segmentation / encode / token
 * counts keep reporting this rank's rows.  on = 0 keeps the sharded exchange to the end.
 * (No reference counterpart: the reference has no multi-GPU path) */
int geobpe_set_collapse(geobpe_ctx *ctx, int on);
/* 1 once the engine has collapsed (then geobpe_step / geobpe_run drive it, as one rank). */
int geobpe_collapsed(geobpe_ctx *ctx);
/* n_merges merges of the row-sharded N > 1 loop with no host wait per merge: per iteration
 * the merge kernels and the records' exchange (the peer exchange above, or the slot export,
 * one all-gather of the fixed slots on the engine's stream and the import); polls every few
 * iterations; a merge whose records overflowed a slot is re-exchanged in full.  A rank runs
 * the middle regime once its share of the winner's count (count / nranks) is below the
 * geobpe_set_mid threshold; the collapse comes below GEOBPE_COLLAPSE_AT (32768) with the peer
 * exchange, below the threshold itself without it.  *n_done = merges made. */
int geobpe_run_exchange(geobpe_ctx *ctx, int64_t n_merges, int64_t *n_done);
/* geobpe_run_exchange with the run's merge records ({new id, count, merged occurrences} per merge,
 * as geobpe_run_log; the reference's BPE._tokens / step log, bpe.py:1857-1866) pulled inside the
 * run's last synchronisation.  *first = the run's first merge index, or -1 when the run went on
 * in the one-rank loop after a collapse (geobpe_merge_log then has them). */
int geobpe_run_exchange_log(geobpe_ctx *ctx, int64_t n_merges, int64_t *n_done, int64_t *first, int64_t *h_out,
                            int64_t cap);

#ifdef __cplusplus
}
#endif
#endif
