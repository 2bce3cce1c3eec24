/*
 * ocffm.h — C ABI of the MI355X-native one-class FFM trainer.
 *
 * This is the drop-in boundary for the reference's hot path (one training
 * epoch of block Newton-CG, johncreed/one-class-ffm ffm.cpp:852-870).  The
 * reference exposes it only as C++ classes (ffm.h:42-154: Parameter, ImpData,
 * ImpProblem, save_model) driven by train.cpp:169-207.  Each entry point
 * below names the reference interface it replaces.  Plain pointers and
 * sizes only: no C++ types, no exceptions, no torch types cross this ABI.
 *
 * All functions return an int status (OCFFM_OK == 0).  On failure,
 * ocffm_last_error() returns a thread-local message.  A problem object is
 * not re-entrant; one host thread drives it.  Device memory is owned by the
 * problem object; host arrays passed in are copied (the caller keeps them).
 */
#ifndef OCFFM_H
#define OCFFM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OCFFM_OK 0
#define OCFFM_E_ARG 1   /* invalid argument   (reference: std::invalid_argument, train.cpp:201-205) */
#define OCFFM_E_IO 2    /* file not readable / not writable                                         */
#define OCFFM_E_DATA 3  /* malformed input (reference: UB, e.g. label >= #items, ffm.cpp:267,382)   */
#define OCFFM_E_HIP 4   /* HIP runtime error, or no GPU                                             */
#define OCFFM_E_COMM 5  /* RCCL error                                                               */
#define OCFFM_E_STATE 6 /* call out of order (e.g. epoch before init)                               */

/* Precision of the device path. */
#define OCFFM_FP64 64 /* parity mode: same arithmetic type as the reference (ffm.h:34-35) */
#define OCFFM_FP32 32 /* perf mode: fp32 tables, fp64 CG scalars and reductions           */

/* Replaces class Parameter (ffm.h:42-49).  Defaults (ocffm_param_default)
 * are the reference's *code* defaults: omega 0.1, lambda 1e-5, r -1,
 * nr_pass 20, k 4, nr_threads 1, self_side 1, freq 0. */
typedef struct ocffm_param {
  double omega;        /* -w : weight of the implicit negatives          */
  double lambda;       /* -l : L2 regularisation                          */
  double r;            /* -r : target value of the negatives              */
  uint32_t nr_pass;    /* -t : epochs                                     */
  uint32_t k;          /* -k : latent dimension (any k in 1..128)         */
  uint32_t nr_threads; /* -c : host threads (parsing); device path ignores */
  int32_t self_side;   /* !--ns : include same-side field-pair blocks     */
  int32_t freq;        /* --freq : lambda scaled by feature frequency     */
  int32_t precision;   /* OCFFM_FP64 or OCFFM_FP32                        */
  int32_t device;      /* HIP device ordinal                              */
} ocffm_param;

void ocffm_param_default(ocffm_param *p);

const char *ocffm_last_error(void);
int ocffm_device_count(int *count);

/* ------------------------------------------------------------------ data
 * Replaces class ImpData (ffm.h:51-79).  A data set is rows of
 * (fid, idx, val) feature nodes plus, for train/test files, a label list of
 * positive item ids per row. */
typedef struct ocffm_data ocffm_data;

typedef struct ocffm_data_info {
  uint64_t m;     /* rows (lines)                                  */
  uint64_t n;     /* max label + 1 (0 for item files)              */
  uint64_t f;     /* fields: max fid + 1 over every token          */
  uint64_t nnz_x; /* kept feature nodes                            */
  uint64_t nnz_y; /* labels                                        */
} ocffm_data_info;

/* ImpData::read + ImpData::split_fields (ffm.cpp:80-257).  With ds != NULL
 * (the train set's per-field Ds, as for test files, train.cpp:191) a node
 * with idx >= ds[fid] is dropped. */
int ocffm_data_read(const char *path, int has_label, const uint64_t *ds, uint32_t nds, ocffm_data **out);

/* The same from in-memory rows: xptr[m+1] row pointers into fid/idx/val,
 * yptr[m+1]/ycol labels (both NULL for an item file). */
int ocffm_data_from_rows(uint64_t m, const uint64_t *xptr, const uint32_t *fid, const uint64_t *idx,
                         const double *val, const uint64_t *yptr, const uint64_t *ycol, const uint64_t *ds,
                         uint32_t nds, ocffm_data **out);

/* ImpData::transY (ffm.cpp:259-294): item-major positives of V from the
 * user-major labels of U. */
int ocffm_data_trans_y(ocffm_data *V, const ocffm_data *U);

int ocffm_data_get_info(const ocffm_data *d, ocffm_data_info *out);
/* Per-field Ds (ffm.cpp:221); out must hold info.f values. */
int ocffm_data_get_ds(const ocffm_data *d, uint64_t *out);
/* The parsed labels (ffm.cpp:93-101: U->Y before transY): yptr holds info.m+1
 * offsets, ycol info.nnz_y item indices.  Either pointer may be NULL. */
int ocffm_data_get_labels(const ocffm_data *d, uint64_t *yptr, uint64_t *ycol);
/* One field's CSR after split_fields (ffm.cpp:185-257): xptr info.m+1
 * offsets, then that field's node indices and values.  Pointers may be NULL;
 * *nnz receives the field's node count. */
int ocffm_data_get_field(const ocffm_data *d, uint32_t field, int64_t *xptr, uint32_t *xidx, double *xval,
                         uint64_t *nnz);
void ocffm_data_free(ocffm_data *d);

/* --------------------------------------------------------------- problem
 * Replaces class ImpProblem (ffm.h:82-151). */
typedef struct ocffm_problem ocffm_problem;

/* ImpProblem(U, Uva, V, param) (ffm.h:84-86).  Ut may be NULL (no -p).  The
 * data sets are copied to the device; V must have been through
 * ocffm_data_trans_y.  Single process, one GPU. */
int ocffm_problem_create(const ocffm_data *U, const ocffm_data *Ut, const ocffm_data *V, const ocffm_param *p,
                         ocffm_problem **out);

/* Data-parallel variant (no reference counterpart: the reference is one
 * process).  One process per GPU; training rows (users) are split into
 * nranks contiguous shards and this rank keeps shard `rank`.  Gradient and
 * Hessian-vector partial sums are all-reduced with RCCL.
 * comm_id: OCFFM_COMM_ID_BYTES bytes from ocffm_comm_id() on rank 0,
 * broadcast by the caller (with nranks == 1 the RCCL path still runs: a
 * one-rank communicator, used by the tests).  Test rows (Ut) are sharded
 * the same way. */
#define OCFFM_COMM_ID_BYTES 128
int ocffm_comm_id(void *out);
int ocffm_problem_create_dist(const ocffm_data *U, const ocffm_data *Ut, const ocffm_data *V,
                              const ocffm_param *p, int rank, int nranks, const void *comm_id,
                              ocffm_problem **out);

/* Host-side all-reduce hook (tests and environments without RCCL).  When
 * set, every sum-all-reduce is staged through host memory and handed to
 * fn(buf, count, is_double, user).  Must be set before ocffm_problem_init. */
typedef int (*ocffm_allreduce_fn)(void *buf, uint64_t count, int is_double, void *user);
int ocffm_problem_create_dist_host(const ocffm_data *U, const ocffm_data *Ut, const ocffm_data *V,
                                   const ocffm_param *p, int rank, int nranks, ocffm_allreduce_fn fn,
                                   void *user, ocffm_problem **out);

/* ImpProblem::init (ffm.cpp:467-512).  W/H are drawn on the host from the
 * C library rand() stream exactly as the reference does (ffm.cpp:71-78).
 * The reference's init is the first rand() consumer of its process (implicit
 * seed 1); HIP runtime start-up in ocffm_problem_create may draw from the
 * stream, so call srand(1) right before this for reference-identical W/H. */
int ocffm_problem_init(ocffm_problem *p);

/* ImpProblem::one_epoch (ffm.cpp:852-870). */
int ocffm_problem_one_epoch(ocffm_problem *p);

/* ImpProblem::solve_side / solve_cross for one block (ffm.cpp:815-850). */
int ocffm_problem_solve_block(ocffm_problem *p, uint32_t f1, uint32_t f2);

/* ImpProblem::cache_sasb (ffm.cpp:514-535). */
int ocffm_problem_cache_sasb(ocffm_problem *p);

/* ImpProblem::solve (ffm.cpp:1147-1161): nr_pass epochs, validation and the
 * stdout table every 10th epoch when a test set is present. */
int ocffm_problem_solve(ocffm_problem *p);

/* ImpProblem::validate (ffm.cpp:925-1016): loss = sqrt(ploss/m_te), p@k and
 * nDCG@k at k = 5,10,20,40,80. */
typedef struct ocffm_metrics {
  double loss;
  double prec[5];
  double ndcg[5];
  uint32_t top_k[5];
} ocffm_metrics;
int ocffm_problem_validate(ocffm_problem *p, ocffm_metrics *out);
/* The reference's nDCG known-answer build (-DEBUG_nDCG -DSHOW_SCORE_ONLY,
 * script/nDCG_degub_tool/readme:1-4): validate() with every test row's
 * scores forced to z_j = n - j after its ploss term (ffm.cpp:988-993).
 * per_row_ndcg (optional, room for cap doubles): nDCG@5,10,20,40,80 of each
 * of this rank's test rows, row-major (ffm.cpp:1059-1128; the build prints
 * the @10 value per row, ffm.cpp:1126).  OCFFM_E_ARG when cap < 5 x
 * ocffm_problem_test_rows(). */
int ocffm_problem_validate_forced(ocffm_problem *p, ocffm_metrics *out, double *per_row_ndcg, uint64_t cap);
/* Test rows of this rank (Uva->m of the reference, ffm.cpp:925; 0 without a
 * test set). */
int ocffm_problem_test_rows(ocffm_problem *p, uint64_t *m);

/* print_epoch_info (ffm.cpp:1130-1145) of the last validation, and the
 * header of init_va (ffm.cpp:901-912), to stdout. */
int ocffm_print_header(void);
int ocffm_print_epoch(const ocffm_metrics *m, uint32_t iter);

/* State access (copies to host as fp64).  what: 'W','H','P','Q' (block
 * b12 = index_vec(f1,f2,f), ffm.cpp:53-55), 'a','b' (biases), 's','t'
 * (sa, sb), 'u' (user-major y-tilde), 'v' (item-major y-tilde).  Returns
 * the element count in *len; copies min(cap, count) values when out != 0.
 * Under sharding, row-indexed user-side arrays are this rank's rows. */
int ocffm_problem_get(ocffm_problem *p, char what, uint32_t b12, double *out, uint64_t cap, uint64_t *len);
/* Overwrite W or H of block b12 (P/Q are recomputed); for tests. */
int ocffm_problem_set(ocffm_problem *p, char what, uint32_t b12, const double *in, uint64_t len);

/* Kernel-level entry points for parity tests.  Gradient of one half
 * (gd_side / gd_cross, ffm.cpp:537-592, 630-703) and lam*v + H(v) of one
 * half (the product inside cg(), ffm.cpp:783-801).  half 0 = W of block
 * (f1,f2), half 1 = H.  Neither changes the solver state. */
int ocffm_problem_grad(ocffm_problem *p, uint32_t f1, uint32_t f2, int half, double *out);
int ocffm_problem_hv(ocffm_problem *p, uint32_t f1, uint32_t f2, int half, const double *v, double *out);

/* save_model (ffm.cpp:1163-1237): the reference's text model format. */
int ocffm_problem_save_model(ocffm_problem *p, const char *path);

/* ImpProblem::save_binary_model (ffm.cpp:1239-1267): W and H of every used
 * block in the reference's binary layout (uint32 f, fu, fv, k; uint64 Ds;
 * per block uint32 index_vec, uint64 |W|, uint64 |H|, doubles). */
int ocffm_problem_save_binary(ocffm_problem *p, const char *path);
/* ImpProblem::load_binary_model (ffm.cpp:1269-1301) as it was meant to work
 * (the reference's opens an ofstream and writes): reads that layout, checks
 * f/fu/fv/k/Ds against this problem, restores W/H and re-derives P, Q, the
 * biases, sa/sb and y-tilde as ocffm_problem_init does.  May replace init. */
int ocffm_problem_load_binary(ocffm_problem *p, const char *path);

/* Statistics.  cg: CG iteration count of every half solved since the last
 * reset (solve order).  Kernel timing is recorded with HIP events on the
 * solver's stream when profiling is on. */
typedef struct ocffm_kernel_stat {
  char name[32];
  uint64_t launches;
  double total_ms;     /* summed event-measured duration        */
  double alg_bytes;    /* summed algorithmic bytes  */
  double alg_flops;    /* summed floating-point ops (MFMA kernels; else 0) */
} ocffm_kernel_stat;
int ocffm_problem_cg_log(ocffm_problem *p, int32_t *out, int cap, int *count);
int ocffm_problem_set_profiling(ocffm_problem *p, int on);
/* Restrict event timing to the kernel family `name` (NULL or "" = all). */
int ocffm_problem_set_profile_filter(ocffm_problem *p, const char *name);
int ocffm_problem_kernel_stats(ocffm_problem *p, ocffm_kernel_stat *out, int cap, int *count);
int ocffm_problem_reset_stats(ocffm_problem *p);
/* Algorithmic HBM bytes of the epochs run since the last reset
 * (SURVEY §8d formula with the actual CG counts). */
int ocffm_problem_alg_bytes(ocffm_problem *p, double *bytes);
/* Diagnostic event counters since create (no reference counterpart):
 * "cgp_launches" (persistent CG launches: column-Gram and id-like side
 * halves), "cgp_side_launches" (the latter), "cgp_side_full" (side halves
 * whose gradient and update ran inside the launch), "cgp_recovered"
 * (launches whose grid gave up on its barrier and whose solve was finished
 * per step), "cgp_refused" (cooperative launches the runtime refused).
 * An unknown name reads 0. */
int ocffm_problem_counter(ocffm_problem *p, const char *name, int64_t *value);
int ocffm_problem_sync(ocffm_problem *p);
/* Digests (FNV-1a over the bytes) of every array of the device data layout
 * the problem built from its ImpData (per-field CSR of split_fields,
 * ffm.cpp:185-257; the item-major positives of transY, ffm.cpp:259-294; the
 * popularity, ffm.cpp:143,172-176; the CSCs, jobs and segments), in a fixed
 * order.  The layout is built on the device unless OCFFM_HOST_BUILD=1 was
 * set at create; both builds give the same digests.  names: cap x 48 chars
 * (may be NULL); *count receives the number of entries. */
int ocffm_problem_layout_digest(ocffm_problem *p, char *names, uint64_t *digests, int cap, int *count);
void ocffm_problem_destroy(ocffm_problem *p);

/* ------------------------------------------------------------ SGD mode
 * BASELINE.json north_star extras, NO reference counterpart (the reference
 * trains only by block Newton-CG): field-aware FM trained per instance by
 * SGD / AdaGrad with lock-free (HOGWILD) writes to W, each positive
 * (user row, item row) of U drawing `nneg` negatives on the device from an
 * alias table over item popularity^neg_power; log-loss.  Instance nodes =
 * the user row's nodes then the item row's (global feature id = field
 * offset + idx).  Parity against oracle/sgd_oracle.cpp (a serial CPU
 * statement), not against the reference ("parity unpinned"). */
typedef struct ocffm_sgd ocffm_sgd;
typedef struct ocffm_sgd_param {
  uint32_t k;          /* latent dimension (1..128)                         */
  float eta;           /* learning rate (libffm default 0.2)                */
  float lambda;        /* L2 (libffm default 2e-5)                          */
  uint32_t nneg;       /* sampled negatives per positive                    */
  double neg_power;    /* alias weights = item label count ^ neg_power      */
  int32_t adagrad;     /* 1: AdaGrad (G starts at 1), 0: plain SGD          */
  int32_t norm;        /* 1: instance-wise 1/|x|^2 normalisation            */
  int32_t serial;      /* 1: one wave, instances in order (parity tests)    */
  uint64_t seed;       /* W init, instance order, negative draws            */
  int32_t device;
} ocffm_sgd_param;
typedef struct ocffm_sgd_info {
  uint64_t n_features; /* NF: rows of W (all fields)      */
  uint32_t n_fields;   /* F                               */
  uint32_t kp;         /* padded row length               */
  uint64_t positives;  /* this rank's positives           */
  uint64_t instances;  /* per epoch: positives (1 + nneg) */
} ocffm_sgd_info;
void ocffm_sgd_param_default(ocffm_sgd_param *p);
int ocffm_sgd_create(const ocffm_data *U, const ocffm_data *V, const ocffm_sgd_param *p, ocffm_sgd **out);
/* One process per GPU: this rank trains on its contiguous user shard's
 * positives; ocffm_sgd_average() makes W and G the mean over the ranks
 * (RCCL all-reduce over xGMI) — periodic model averaging. */
int ocffm_sgd_create_dist(const ocffm_data *U, const ocffm_data *V, const ocffm_sgd_param *p, int rank, int nranks,
                          const void *comm_id, ocffm_sgd **out);
/* The same with ocffm_sgd_average's sums staged through host memory and
 * handed to fn (float arrays: W, then G) — tests of the sharding on one GPU. */
int ocffm_sgd_create_dist_host(const ocffm_data *U, const ocffm_data *V, const ocffm_sgd_param *p, int rank,
                               int nranks, ocffm_allreduce_fn fn, void *user, ocffm_sgd **out);
int ocffm_sgd_epoch(ocffm_sgd *s, double *mean_loss);
int ocffm_sgd_average(ocffm_sgd *s);
/* phi for n (user row, item row) pairs with the current W. */
int ocffm_sgd_phi(ocffm_sgd *s, uint64_t n, const uint32_t *users, const uint32_t *items, float *out);
/* what: 'W' / 'G' (float, NF x F x kp), 'p' alias probabilities (float),
 * 'a' alias targets (uint32), 'o' last epoch's order (uint64 A, B, T). */
int ocffm_sgd_get(ocffm_sgd *s, char what, void *out, uint64_t cap, uint64_t *len);
int ocffm_sgd_set_w(ocffm_sgd *s, const float *w, uint64_t n);
int ocffm_sgd_get_info(ocffm_sgd *s, ocffm_sgd_info *out);
int ocffm_sgd_sync(ocffm_sgd *s);
void ocffm_sgd_destroy(ocffm_sgd *s);

#ifdef __cplusplus
}
#endif
#endif /* OCFFM_H */
