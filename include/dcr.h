/*
 * dcr.h — C-ABI of the MI355X duplex-consensus hot path (libdcr.so).
 *
 * Replaces, per batch of MI families, the six calls per family the reference
 * makes to
 *     make_consensus_read(list_of_reads, method)
 *         /root/reference/DuplexUMIConsensusReads.py:1291-1386
 * (4x method="single_strand" at :1569, 2x method="double_strand" at :1581-1582)
 * together with the per-read preprocessing they consume
 *     remove_clipping / mask_low_quality_bases / trim_3prime_N   :191-325
 * The reference has no FFI of its own (it is one Python script whose config
 * is module globals, :1432-1469); INTEGRATION.md shows the ctypes binding the
 * host uses (duplexumiconsensusreads_amd/_lib.py) and how a maintainer would
 * call it from the reference's main() loop (:1560-1588).
 *
 * Plain pointers and sizes only.  All batch/out pointers passed to
 * dcr_run_batch are DEVICE pointers (HBM-resident inputs); dcr_run_batch_host
 * takes HOST pointers and stages through the context's device buffers.
 * Errors: functions return 0 or a DCR_E* code; the message is available from
 * dcr_last_error() (thread-local).  Per-record "the reference would raise"
 * outcomes are reported in the status arrays, not as errors.
 */
#ifndef DCR_H
#define DCR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DCR_ABI_VERSION 1
#define DCR_LUT_PLUS 256   /* LUT row of '+' (absence of insertion), :667-669 */
#define DCR_LUT_DEL 257    /* LUT row of '-' (deletion), :670-672            */
#define DCR_LUT_N 258
#define DCR_MAX_QTHRESH 257

/* return codes */
enum {
    DCR_OK = 0,
    DCR_EARG = 1,       /* bad argument / params                                */
    DCR_EHIP = 2,       /* HIP runtime error                                    */
    DCR_ECAPACITY = 3,  /* an output region is smaller than the consensus needs */
    DCR_ENODEV = 4      /* no usable gfx950 device                              */
};

/* per-record status (what the reference does on these inputs) */
enum {
    DCR_ST_OK = 0,
    DCR_ST_INDEX_ERROR = 1,    /* IndexError: compress_cigarlist([]) :740, insertion past
                                  the sequence end :485                               */
    DCR_ST_TYPE_ERROR = 2,     /* TypeError: a read/consensus without sequence (:402)  */
    DCR_ST_VALUE_ERROR = 3,    /* ValueError: max() of an empty depth list (:1005)     */
    DCR_ST_OVERFLOW_ERROR = 4, /* OverflowError: quality outside uint8 (:1383)         */
    DCR_ST_EXIT_BADCHAR = 5,   /* sys.exit(1): invalid nucleotide (:582-585)           */
    DCR_ST_UPSTREAM = 6,       /* duplex, not computed: an input consensus failed      */
    DCR_ST_PREP = 0x10         /* single-strand: DCR_ST_PREP | s = the preprocessing of a read
                                  raised s (the subfamily's first failing read, :1272-1283) */
};

/* context options (dcr_set_options) */
#define DCR_OPT_READ_INFO 1    /* every read's dcr_read_info is written (parity tests; costs
                                  24 B of HBM writes per read); otherwise only failing reads' */

/* Numeric flags (:1432-1469) plus host-built tables.  The tables are built on
 * the host with the reference's own Python arithmetic (params.py), so the
 * device never evaluates pow/log10 (bit-exact by construction). */
typedef struct dcr_params {
    int32_t min_base_quality;        /* --min_base_quality (seqQ_threshold)   */
    int32_t max_base_quality;        /* --max_base_quality                    */
    int32_t base_quality_shift;      /* --base_quality_shift                  */
    int32_t error_rate_post_labeling;/* --error_rate_post_labeling (raw int)  */
    int32_t error_rate_pre_labeling; /* --error_rate_pre_labeling (raw int)   */
    int32_t deletion_score;          /* --deletion_score                      */
    int32_t no_insertion_score;      /* --no_insertion_score                  */
    int32_t n_qthresh;               /* entries used in qthresh (= maxQ + 1)  */
    /* (1 - p') and p'/5 for quality codes 0..255, '+' (256), '-' (257);
       p' = post*(1-ps) + (1-post)*ps + post*ps*4/5, ps = 10**(-s/10)  :665-676 */
    double match[DCR_LUT_N];
    double mismatch[DCR_LUT_N];
    double post_threshold;           /* 1 - 10**(-min_base_quality/10)   :679-680 */
    /* qthresh[i] = smallest double x > 0 with int(round(-10*log10(x), 0)) <= i-1,
       i = 0..maxQ (decreasing in i).  For a finite error x > 0 the consensus
       quality (:699-709) is Q = maxQ - #{i : x >= qthresh[i]}; Q < 0 means the
       reference would store a negative quality (OverflowError).  x <= 0 or NaN
       give maxQ (the reference's ValueError branch). */
    double qthresh[DCR_MAX_QTHRESH];
} dcr_params;

/* One batch of families, struct-of-arrays.  Subfamily s = 4*f + k with
 * k = 0..3 for A1, B2, B1, A2 (split_family :132-154); reads of a subfamily
 * are contiguous and in reference order (after check_number_reads' random
 * downsampling, :157-188, which stays on the host). */
typedef struct dcr_batch {
    int32_t n_fam;
    int32_t n_reads;
    int64_t n_cigar;            /* entries of cigar                              */
    int64_t n_bases;            /* entries of bases / quals                      */
    int64_t ss_cols;            /* ss_col_off[4F]                                */
    int64_t ds_cols;            /* ds_col_off[2F]                                */
    const int32_t *sub_off;     /* [4F+1] first read of each subfamily          */
    const int32_t *read_pos;    /* [n_reads] reference_start (0-based)          */
    const uint8_t *read_mapq;   /* [n_reads] mapping_quality                    */
    const int64_t *seq_off;     /* [n_reads] offset into bases/quals            */
    const int32_t *seq_len;     /* [n_reads] query length incl. soft clips      */
    const int32_t *cig_off;     /* [n_reads] offset into cigar                  */
    const int32_t *cig_n;       /* [n_reads] number of cigar ops                */
    const uint32_t *cigar;      /* BAM encoding (len << 4 | op)                 */
    const uint8_t *bases;       /* ASCII bases as stored (before masking)       */
    const uint8_t *quals;       /* phred qualities                              */
    const int64_t *ss_col_off;  /* [4F+1] single-strand output region offsets   */
    const int64_t *ds_col_off;  /* [2F+1] duplex output region offsets          */
} dcr_batch;

/* Results of one consensus kind (single-strand: 4F records, duplex: 2F).
 * Variable-length fields live in the record's region [col_off[i], col_off[i+1]). */
typedef struct dcr_out {
    uint8_t *status;    /* DCR_ST_*                                            */
    int32_t *pos;       /* consensus reference_start (:790)                    */
    int32_t *mapq;      /* trunc(mean(mapq)) (:874-889, :1377)                 */
    int32_t *len;       /* consensus sequence length                           */
    int32_t *n_cig;     /* consensus cigar ops                                 */
    int32_t *n_de;      /* entries of d / e (:1002-1003)                       */
    int32_t *D;         /* max depth                                           */
    int32_t *M;         /* min depth                                           */
    double *E;          /* round(mean(e/d), 3)                                 */
    uint8_t *seq;       /* ASCII consensus bases                               */
    uint8_t *qual;      /* consensus qualities                                 */
    uint32_t *cigar;    /* BAM encoding                                        */
    uint16_t *d;        /* per-column depth                                    */
    uint16_t *e;        /* per-column errors                                   */
} dcr_out;

/* Per-read preprocessing results (exported so the host can rebuild the
 * preprocessed input records the reference would tag; optional). */
typedef struct dcr_read_info {
    int64_t seq_start;  /* offset of the first kept base (after 5' soft clip)  */
    int32_t len;        /* kept length after 3' N trim                         */
    int32_t n_cig;      /* normalised cigar ops (M/I/D only)                   */
    int32_t status;     /* DCR_ST_*                                            */
    int32_t has_ins;    /* any I op kept                                       */
} dcr_read_info;

typedef struct dcr_ctx dcr_ctx;

/* library */
int dcr_abi_version(void);
const char *dcr_last_error(void);

/* context: one per GPU (not thread-safe per context) */
dcr_ctx *dcr_create(int device, const dcr_params *params);
void dcr_destroy(dcr_ctx *ctx);
int dcr_set_params(dcr_ctx *ctx, const dcr_params *params);
int dcr_set_options(dcr_ctx *ctx, int flags);   /* DCR_OPT_* */
/* pre-size internal scratch so a timed loop never allocates */
int dcr_reserve(dcr_ctx *ctx, const dcr_batch *sizes);
void *dcr_stream(dcr_ctx *ctx);   /* the context's hipStream_t */

/* device-pointer batch: asynchronous on the context stream */
int dcr_run_batch(dcr_ctx *ctx, const dcr_batch *in, dcr_out *ss, dcr_out *ds);
/* host-pointer batch: stages H2D, runs, D2H; synchronous */
int dcr_run_batch_host(dcr_ctx *ctx, const dcr_batch *in, dcr_out *ss, dcr_out *ds);
int dcr_sync(dcr_ctx *ctx);
/* copy the last batch's per-read preprocessing info (host pointer, n_reads);
   complete only with DCR_OPT_READ_INFO */
int dcr_read_info_host(dcr_ctx *ctx, dcr_read_info *out, int64_t n_reads);
/* timing of the last dcr_run_batch (HIP events on the context stream), ms:
   [0] prep (always 0: fused into the consensus kernels), [1] single-strand,
   [2] duplex, [3] whole batch */
int dcr_last_timing(dcr_ctx *ctx, float *ms4);
/* per-kernel timing of the last dcr_run_batch (HIP events between launches on
   the context stream), ms: per strand (single-strand, duplex) k_recmeta,
   k_consensus_fast, k_consensus_fast (exact queue), k_consensus_general */
#define DCR_N_KERNEL_TIMES 8
int dcr_last_kernel_timing(dcr_ctx *ctx, float *ms8);

/* Streaming: a context has DCR_MAX_SLOTS slots of device buffers.
 * dcr_submit copies a host batch (pinned memory, dcr_host_alloc) into the
 * slot on a copy stream, runs it on the compute stream and copies the
 * outputs back into the host dcr_out arrays on a second copy stream (NULL
 * fields are not copied); it returns at once.  read_status (optional,
 * n_reads int32) receives dcr_read_info.status of every read.  dcr_wait
 * blocks until the slot's outputs are on the host.  Batches run on the
 * device in submission order; H2D of one batch and D2H of another overlap
 * the kernels of a third. */
#define DCR_MAX_SLOTS 4
void *dcr_host_alloc(size_t bytes);
void dcr_host_free(void *p);
int dcr_submit(dcr_ctx *ctx, int slot, const dcr_batch *host_in, dcr_out *host_ss, dcr_out *host_ds,
               int32_t *read_status);
int dcr_wait(dcr_ctx *ctx, int slot);

/* Device record writer.  dcr_submit_write is dcr_submit followed, on the
 * device, by the reference's per-family outcome (what make_consensus_read /
 * preprocess_family raise, in its order), the two duplex BAM records of every
 * family that does not fail (make_consensus_read :1352-1384, add_tags
 * :1076-1120, fix_paired_end_fields :1390-1419), formatted as the host writer
 * (libdcr_io dcr_fmt_write) formats them, and their BGZF compression; only
 * the compressed blocks, the outcomes and the duplex lengths come back.
 * dcr_wait_write waits for the slot and copies the blocks into res->bgzf.
 * The formatted records stay in the slot until it is submitted again
 * (dcr_slot_fetch: what 0 = record bytes, 1 = int64 record offsets [2F+1],
 * 2 = the BGZF blocks again, e.g. after dcr_wait_write found cap_bgzf too
 * small: totals[0] holds the size). */
typedef struct dcr_wmeta {
    const char *names;           /* string arena (dcr_host_batch.names)          */
    int64_t n_names;
    const int64_t *fam_code;     /* [F] offsets of the family codes (MI prefix)  */
    const int64_t *fam_rx;       /* [2F] offsets of RX of the A1 / B1 read0      */
    const int32_t *fam_tid;      /* [F] reference_id                             */
} dcr_wmeta;
typedef struct dcr_wres {        /* pinned host memory                          */
    uint8_t *bgzf;               /* BGZF blocks of the batch's records, in order */
    int64_t cap_bgzf;
    int32_t *fam_fail;           /* [F] DCR_FAIL_* | which << 8 (include/dcr_io.h), 0: written */
    int32_t *ds_len;             /* [2F] duplex consensus lengths                */
    int64_t *totals;             /* [3] BGZF bytes, record bytes, BGZF blocks    */
} dcr_wres;
int dcr_submit_write(dcr_ctx *ctx, int slot, const dcr_batch *host_in, const dcr_wmeta *meta, dcr_wres *res);
int dcr_wait_write(dcr_ctx *ctx, int slot, dcr_wres *res);
int dcr_slot_fetch(dcr_ctx *ctx, int slot, int what, int64_t off, int64_t n, void *dst);

/* CPU restatement with the same contract (oracle/, test infrastructure):
   host pointers, single thread (or n_threads > 1) */
int dcr_oracle_run(const dcr_params *params, const dcr_batch *in, dcr_out *ss, dcr_out *ds,
                   dcr_read_info *info, int n_threads);

#ifdef __cplusplus
}
#endif
#endif /* DCR_H */
