// dcr_capi.hip — C-ABI of libdcr.so (include/dcr.h): context, workspace,
// launches and timing for the gfx950 kernels in dcr_kernels.hip.
//
// One context per GPU: its own HIP stream, device copy of the parameters, and
// a grow-only workspace (reserve it once; the launch path never allocates,
// so a caller may capture dcr_run_batch into a hipGraph).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstddef>
#include <cstring>
#include <cstdlib>
#include <string>
#include <vector>

#include "dcr_internal.h"
#include "dcr_deflate.h"
#include "dcr_writer.h"

namespace {
thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                  \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess)                                                          \
            return fail(DCR_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(&p, n ? n : 16);
        if (e == hipSuccess) cap = n;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }
}  // namespace

int dcr::set_error(int code, const std::string &msg) { return fail(code, msg); }

// The batch streams run at the device's highest priority: the input
// inflater's long launches (include/dcr_inflate.h) share the GPU and a
// batch's kernels should not queue behind spans inflated far ahead.
static hipError_t hi_prio_stream(hipStream_t *s) {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = 0;
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest);
}

struct dcr_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // ev[0] batch start, ev[1..8] after k_recmeta<ss>, fast<ss>, exact<ss>, general<ss>,
    // k_recmeta<ds>, fast<ds>, exact<ds>, general<ds>
    hipEvent_t ev[DCR_N_KERNEL_TIMES + 1] = {};
    dcr_params *d_params = nullptr;
    DevBuf ws;          // workspace
    DevBuf io;          // staging for the host-pointer entry point
    // streaming (dcr_submit / dcr_wait): copy streams and per-slot device buffers
    hipStream_t s_h2d = nullptr, s_d2h = nullptr;
    // dcr_wait_write's copy of the compressed blocks: a stream of its own, so
    // that it does not queue behind the next batch's downloads on s_d2h
    // (which wait for that batch's kernels)
    hipStream_t s_fetch = nullptr;
    hipEvent_t ev_fetch = nullptr;      // blocking-sync event after the compressed-block copy
    struct Slot {
        DevBuf buf;
        DevBuf wbuf;              // device record writer: metadata, record stream, BGZF blocks
        int64_t *d_rec_off = nullptr, *d_comp_n = nullptr;
        uint8_t *d_stream = nullptr, *d_comp = nullptr;
        int64_t n_fam = 0;
        bool writer = false;
        hipEvent_t ev_h2d = nullptr, ev_comp = nullptr, ev_d2h = nullptr;
        int *h_err = nullptr;     // pinned copy of the batch's capacity flag
        bool busy = false;
    } slots[DCR_MAX_SLOTS];
    dcr::Workspace w{};
    int64_t last_reads = 0;
    bool timed = false;
    int fast_ok = 0;    // fast_allowed(): the fast kernel may take records
    int options = 0;    // DCR_OPT_*
    int wide_ok = 0;    // the general kernel's decision pass may run (wide_table)
    dcr_params host_params{};
    // fast-kernel constants (fast_constants)
    uint32_t fast_kq = 0, fast_kqlo = 0;
    int fast_maxq = 0, fast_t16 = 0, fast_r_safe = 0, fast_qlo = 0;
    int fast_t8 = 0, fast_narrow = 0;   // the common fast instantiation's narrow rows (1/8 nat)
    // single-strand records of at most this many reads skip the common fast
    // pass (the exact pass takes them whole); DCR_EXACT_DIRECT_R overrides
    int direct_r = 3;
    // the largest single-strand subfamily of the batch being submitted, when
    // the host knows it (dcr_submit / dcr_submit_write: host sub_off), else -1:
    // the kernels only records that large can need (k_prep_big > 64 reads,
    // k_decide_deep >= kDeepReads) are not launched for batches without them
    int max_r_hint = -1;
    int rm_waves = dcr::kRecmetaWaves;   // k_recmeta block size for light records (DCR_RM_WAVES: A/B runs)
    uint16_t *d_llr16 = nullptr;   // device [128]
    uint16_t *d_llr8 = nullptr;    // device [128]
    uint32_t *d_r2tab = nullptr;   // device [dcr::kR2Entries]: two-read column outcomes (EXACT pass)
    double *d_e1000 = nullptr;     // device [1001]: k / 1000 (the fast kernel's E)
    uint32_t *d_wtab = nullptr;    // device [DCR_LUT_N] (general kernel's decision pass)
    int n_cu = 256;     // compute units (persistent grid size)
    int dfl_blocks = 1; // resident k_deflate workgroups per CU (dynamic LDS = sizeof(dfl::Shared))
    int fast_blocks[4] = {1, 1, 1, 1};   // resident k_consensus_fast blocks per CU (ss, ds; exact ss, exact ds)
};

// The fast kernel's assumptions (dcr_kernels.hip, fast kernel v2): every
// likelihood factor in [0, 1]; the quality formula reduces to e (no pre/post
// labelling error, :700-709); qualities fit a byte (:1383).  Otherwise every
// record takes the general kernel.
static int fast_allowed(const dcr_params *p) {
    for (int i = 0; i < DCR_LUT_N; ++i)
        if (!(p->match[i] >= 0.0 && p->match[i] <= 1.0 && p->mismatch[i] >= 0.0 && p->mismatch[i] <= 1.0))
            return 0;
    return p->error_rate_pre_labeling == 0 && p->error_rate_post_labeling == 0 && p->max_base_quality <= 255 &&
           p->min_base_quality <= 255;
}

// Host constants of the fast kernel's decision (dcr_kernels.hip, fast kernel v6):
//   llr16[q] = floor(16 ln(match[q] / mismatch[q]) - 1e-6)  (a lower bound; + 1 an upper one)
//   t16      = ceil(16 ln(5 / cc)) + 1,  cc = min(qthresh[maxQ], 1 - threshold, 1/4)
//   fast_qlo = the lowest quality from which every row has match >= mismatch > 0
//   r_safe   = the most reads R with R c_max <= 700 nats, c_max bounding -ln of either factor of
//              the rows a fast record can hold (q <= 122; the call's rows have q >= fast_qlo).
//              ln L_b >= -R c_max, so up to r_safe reads the call's likelihood stays a normal
//              double (e^-700 > DBL_MIN = e^-708.4).
//              Above it the reference's products can underflow to 0 (S = 0, NaN posterior, call
//              'A' :613), which the LLR bound does not see: every column then takes the exact path.
//   llrn[q], tn: the same in 1/u nat for the common fast instantiation's
//              narrow rows (dcr_kernels.hip, Evidence8: 15 rows of at most 273
//              fit 12 bits), u = 16 when every row fits (default parameters:
//              qualities capped at max_base_quality 60 give <= 246), else 8, else
//              4; narrow = 0 when none does (then that instantiation queues every
//              record for the EXACT one)
// Returns 0 when the decision cannot be made for these parameters (then every
// record takes the general kernel).
static int fast_constants(const dcr_params &hp, uint16_t llr16[128], uint16_t llr8[128], uint32_t &kq, uint32_t &kqlo,
                          int &maxq, int &t16, int &t8, int &narrow, int &r_safe, int &qlo_out) {
    const int mb = std::min(std::max(hp.min_base_quality, 0), 255);
    kq = (uint32_t)(255 - mb) * 0x01010101u;
    maxq = hp.max_base_quality;
    int qlo = 123;
    while (qlo > 0 && hp.mismatch[qlo - 1] > 0.0 && hp.match[qlo - 1] >= hp.mismatch[qlo - 1]) --qlo;
    kqlo = (uint32_t)(0x80 - qlo) * 0x01010101u;
    qlo_out = qlo;
    double lmax = 0.0;
    for (int q = 0; q < 128; ++q) {
        llr16[q] = 0;
        if (q >= qlo && q <= 122) {
            const double v = std::floor(16.0 * std::log(hp.match[q] / hp.mismatch[q]) - 1e-6);
            if (!(v <= 1040.0)) return 0;                  // 63 rows must fit a 16-bit field
            llr16[q] = (uint16_t)std::max(v, 0.0);
            lmax = std::max(lmax, std::log(hp.match[q] / hp.mismatch[q]));
        }
    }
    // the narrow rows' unit: 15 rows must fit 12 bits
    int un = 16;
    while (un > 4 && std::floor(un * lmax - 1e-6) > 273.0) un /= 2;
    narrow = std::floor(un * lmax - 1e-6) <= 273.0 ? 1 : 0;
    for (int q = 0; q < 128; ++q) {
        llr8[q] = 0;
        if (narrow && q >= qlo && q <= 122)
            llr8[q] = (uint16_t)std::max(std::floor(un * std::log(hp.match[q] / hp.mismatch[q]) - 1e-6), 0.0);
    }
    const int mq = std::min(std::max(hp.max_base_quality, 0), DCR_MAX_QTHRESH - 1);
    const double cc = std::min(std::min(hp.qthresh[mq], 1.0 - hp.post_threshold), 0.25);
    if (!(cc > 1e-12)) return 0;
    t16 = (int)std::ceil(16.0 * std::log(5.0 / cc)) + 1;
    t8 = (int)std::ceil(un * std::log(5.0 / cc)) + 1;
    double cmax = 0.0;                                 // per-row bound on -ln(factor), either factor
    for (int q = 0; q <= 122; ++q) {
        cmax = std::max(cmax, -std::log(hp.mismatch[q]));
        if (q >= qlo) cmax = std::max(cmax, -std::log(hp.match[q]));
    }
    r_safe = cmax > 0.0 ? (int)std::min(1e6, std::floor(700.0 / cmax)) : 1000000;
    return 1;
}

// The general kernel's decision pass (dcr_kernels.hip: decide_record) per LUT
// row v (quality byte, '+' 256, '-' 257):
//   bits 0-15   llr16 = floor(16 ln(match[v] / mismatch[v]) - 1e-6), a lower bound
//   bits 16-30  z16   = ceil(16 (-ln mismatch[v]) + 1e-6), an upper bound
//   bit 31      the row cannot be a call's row (quality above 122 or below fast_qlo; '+' / '-' with 1-p' < p'/5)
// Returns 0 when some z16 does not fit (then the pass is not used).
static int wide_table(const dcr_params &hp, uint32_t wtab[DCR_LUT_N]) {
    int qlo = 123;
    while (qlo > 0 && hp.mismatch[qlo - 1] > 0.0 && hp.match[qlo - 1] >= hp.mismatch[qlo - 1]) --qlo;
    for (int v = 0; v < DCR_LUT_N; ++v) {
        const double mm = hp.mismatch[v], m = hp.match[v];
        if (!(mm > 0.0)) return 0;
        const double z = std::ceil(-16.0 * std::log(mm) + 1e-6);
        if (!(z >= 0.0 && z <= 32767.0)) return 0;
        uint32_t w = (uint32_t)z << 16;
        const bool call_row = v >= DCR_LUT_PLUS ? m >= mm : (v >= qlo && v <= 122);   // '+', '-' rows
        if (call_row) {
            const double l = std::floor(16.0 * std::log(m / mm) - 1e-6);
            if (!(l <= 1040.0)) return 0;
            w |= (uint32_t)std::max(l, 0.0);
        } else {
            w |= 1u << 31;
        }
        wtab[v] = w;
    }
    return 1;
}

static int upload_fast(dcr_ctx *c, const dcr_params *params) {
    uint16_t llr[128], llr8[128];
    uint32_t wtab[DCR_LUT_N];
    const int ok = fast_constants(*params, llr, llr8, c->fast_kq, c->fast_kqlo, c->fast_maxq, c->fast_t16, c->fast_t8,
                                 c->fast_narrow, c->fast_r_safe, c->fast_qlo);
    c->fast_ok = fast_allowed(params) && ok;
    c->wide_ok = c->fast_ok && wide_table(*params, wtab);
    if (hipMemcpy(c->d_llr16, llr, sizeof(llr), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_llr8, llr8, sizeof(llr8), hipMemcpyHostToDevice) != hipSuccess ||
        (c->wide_ok && hipMemcpy(c->d_wtab, wtab, sizeof(wtab), hipMemcpyHostToDevice) != hipSuccess))
        return fail(DCR_EHIP, "fast-kernel table upload failed");
    // the two-read outcomes from the device parameters just uploaded, by the
    // EXACT pass's own products and posterior (bit-identical by construction)
    hipLaunchKernelGGL(dcr::k_r2_table, dim3((dcr::kR2Entries + 255) / 256), dim3(256), 0, c->stream, c->d_params,
                       c->d_r2tab);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess)
        return fail(DCR_EHIP, "two-read table build failed");
    return DCR_OK;
}

extern "C" {

int dcr_abi_version(void) { return DCR_ABI_VERSION; }

const char *dcr_last_error(void) { return g_err.c_str(); }

static int check_params(const dcr_params *p) {
    if (!p) return fail(DCR_EARG, "params is NULL");
    if (p->max_base_quality < 0 || p->max_base_quality > DCR_MAX_QTHRESH - 1)
        return fail(DCR_EARG, "max_base_quality out of range [0, 256]");
    if (p->n_qthresh != p->max_base_quality + 1)
        return fail(DCR_EARG, "n_qthresh must equal max_base_quality + 1");
    return DCR_OK;
}

dcr_ctx *dcr_create(int device, const dcr_params *params) {
    if (check_params(params) != DCR_OK) return nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
        fail(DCR_ENODEV, "no HIP device " + std::to_string(device));
        return nullptr;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess ||
        std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        fail(DCR_ENODEV, std::string("device is not gfx950 (MI355X): ") + prop.gcnArchName);
        return nullptr;
    }
    dcr_ctx *c = new dcr_ctx();
    c->device = device;
    if (const char *e = std::getenv("DCR_EXACT_DIRECT_R")) c->direct_r = std::atoi(e);   // A/B runs
    if (const char *e = std::getenv("DCR_RM_WAVES")) {                                  // A/B runs
        const int w = std::atoi(e);
        if (w == 4 || w == 8 || w == 16) c->rm_waves = w;
    }
    if (hipSetDevice(device) != hipSuccess ||
        hi_prio_stream(&c->stream) != hipSuccess ||
        hipMalloc(&c->d_params, sizeof(dcr_params)) != hipSuccess ||
        hipMalloc(&c->d_llr16, 128 * sizeof(uint16_t)) != hipSuccess ||
        hipMalloc(&c->d_llr8, 128 * sizeof(uint16_t)) != hipSuccess ||
        hipMalloc(&c->d_r2tab, dcr::kR2Entries * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&c->d_e1000, 1001 * sizeof(double)) != hipSuccess ||
        hipMalloc(&c->d_wtab, DCR_LUT_N * sizeof(uint32_t)) != hipSuccess) {
        fail(DCR_EHIP, "context allocation failed");
        delete c;
        return nullptr;
    }
    for (auto &e : c->ev) (void)hipEventCreate(&e);
    (void)hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device);
    // the persistent fast kernel's grid = what is resident at once (a block
    // beyond that would start only when a resident one has finished its range)
    const void *fk[4] = {(const void *)dcr::k_consensus_fast<false, false>, (const void *)dcr::k_consensus_fast<true, false>,
                         (const void *)dcr::k_consensus_fast<false, true>, (const void *)dcr::k_consensus_fast<true, true>};
    for (int k = 0; k < 4; ++k)
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&c->fast_blocks[k], fk[k], dcr::kFastBlock, 0) != hipSuccess ||
            c->fast_blocks[k] < 1)
            c->fast_blocks[k] = 1;
    if (hipFuncSetAttribute((const void *)dcrw::k_deflate, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(dfl::Shared)) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&c->dfl_blocks, dcrw::k_deflate, dfl::kT, sizeof(dfl::Shared)) !=
            hipSuccess ||
        c->dfl_blocks < 1)
        c->dfl_blocks = 1;
    c->host_params = *params;
    double e1000[1001];
    for (int k = 0; k <= 1000; ++k) e1000[k] = (double)k / 1000.0;   // IEEE division: numpy's rint(x)/1000
    if (hipMemcpy(c->d_params, params, sizeof(dcr_params), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_e1000, e1000, sizeof(e1000), hipMemcpyHostToDevice) != hipSuccess ||
        upload_fast(c, params) != DCR_OK) {
        fail(DCR_EHIP, "params upload failed");
        dcr_destroy(c);
        return nullptr;
    }
    return c;
}

void dcr_destroy(dcr_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    c->ws.release();
    c->io.release();
    for (auto &S : c->slots) {
        if (S.ev_d2h) (void)hipEventSynchronize(S.ev_d2h);
        S.buf.release();
        S.wbuf.release();
        if (S.ev_h2d) (void)hipEventDestroy(S.ev_h2d);
        if (S.ev_comp) (void)hipEventDestroy(S.ev_comp);
        if (S.ev_d2h) (void)hipEventDestroy(S.ev_d2h);
        if (S.h_err) (void)hipHostFree(S.h_err);
    }
    if (c->s_h2d) (void)hipStreamDestroy(c->s_h2d);
    if (c->s_d2h) (void)hipStreamDestroy(c->s_d2h);
    if (c->s_fetch) (void)hipStreamDestroy(c->s_fetch);
    if (c->ev_fetch) (void)hipEventDestroy(c->ev_fetch);
    if (c->d_params) (void)hipFree(c->d_params);
    if (c->d_llr16) (void)hipFree(c->d_llr16);
    if (c->d_llr8) (void)hipFree(c->d_llr8);
    if (c->d_r2tab) (void)hipFree(c->d_r2tab);
    if (c->d_e1000) (void)hipFree(c->d_e1000);
    if (c->d_wtab) (void)hipFree(c->d_wtab);
    for (auto &e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int dcr_set_params(dcr_ctx *c, const dcr_params *params) {
    if (!c) return fail(DCR_EARG, "ctx is NULL");
    int rc = check_params(params);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpyAsync(c->d_params, params, sizeof(dcr_params), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->host_params = *params;
    return upload_fast(c, params);
}

void *dcr_stream(dcr_ctx *c) { return c ? (void *)c->stream : nullptr; }

int dcr_set_options(dcr_ctx *c, int flags) {
    if (!c) return fail(DCR_EARG, "ctx is NULL");
    if (flags & ~DCR_OPT_READ_INFO) return fail(DCR_EARG, "unknown option");
    c->options = flags;
    return DCR_OK;
}

int dcr_reserve(dcr_ctx *c, const dcr_batch *s) {
    if (!c || !s) return fail(DCR_EARG, "NULL argument");
    HIP_TRY(hipSetDevice(c->device));
    const int64_t cols = std::max(s->ss_cols, s->ds_cols);
    size_t o = 0;
    const size_t o_info = o; o = align_up(o + sizeof(dcr_read_info) * (size_t)std::max<int64_t>(s->n_reads, 1));
    const size_t o_cig = o;  o = align_up(o + sizeof(uint32_t) * (size_t)std::max<int64_t>(s->n_cigar, 1));
    const size_t o_cons = o; o = align_up(o + sizeof(int32_t) * (size_t)std::max<int64_t>(cols, 1));
    const size_t o_et = o;   o = align_up(o + sizeof(double) * (size_t)std::max<int64_t>(cols, 1));
    const size_t o_ins = o;  o = align_up(o + (size_t)std::max<int64_t>(s->ss_cols, 1));
    const size_t o_st = o;   o = align_up(o + sizeof(int4) * (size_t)std::max<int64_t>(s->n_reads, 1));
    const size_t o_err = o;  o = align_up(o + 64);
    const size_t o_stamp = o; o = align_up(o + 64 * sizeof(unsigned long long));
    const size_t n_rec = (size_t)std::max<int64_t>(4LL * s->n_fam, 1);
    const size_t o_ovf = o;  o = align_up(o + sizeof(int) * n_rec);
    const size_t o_xl = o;   o = align_up(o + sizeof(int) * n_rec);
    const size_t o_deep = o; o = align_up(o + sizeof(int) * n_rec);
    const size_t o_meta = o; o = align_up(o + sizeof(dcr::RecMeta) * n_rec);
    const size_t o_rm = o;   o = align_up(o + sizeof(uint2) * std::max<size_t>((size_t)s->n_reads, n_rec));
    const size_t o_rows = o; o = align_up(o + sizeof(uint4) * n_rec);
    // insertion layouts: a row of kLayRow codes per single-strand read and per
    // duplex input (two per duplex record)
    const size_t o_lb = o;   o = align_up(o + sizeof(int) * (size_t)std::max<int64_t>(6LL * s->n_fam, 1));
    const size_t o_lm = o;   o = align_up(o + 4 * sizeof(uint64_t) * (size_t)std::max<int64_t>(6LL * s->n_fam, 1));
    const size_t o_lay = o;
    o = align_up(o + sizeof(uint16_t) * (size_t)dcr::kLayRow * (size_t)std::max<int64_t>(s->n_reads + 4LL * s->n_fam, 1));
    if (o > c->ws.cap) {
        HIP_TRY(hipStreamSynchronize(c->stream));
        HIP_TRY(c->ws.ensure(o + o / 8));
    }
    char *b = (char *)c->ws.p;
    c->w.info = (dcr_read_info *)(b + o_info);
    c->w.norm_cig = (uint32_t *)(b + o_cig);
    c->w.cons = (int32_t *)(b + o_cons);
    c->w.et = (double *)(b + o_et);
    c->w.insflag = (uint8_t *)(b + o_ins);
    c->w.state = (int4 *)(b + o_st);
    c->w.err = (int *)(b + o_err);
    c->w.ovf_count = (int *)(b + o_err) + 1;     // err, ovf_count[2], fast_count[2], xcount[2], gen_next[2]: one block
    c->w.fast_count = (int *)(b + o_err) + 3;
    c->w.xcount = (int *)(b + o_err) + 5;
    c->w.gen_next = (int *)(b + o_err) + 7;      // [2], in the same block: reset with it per batch
    c->w.deep_count = (int *)(b + o_err) + 9;    // [1], likewise
    c->w.lay_next = (int *)(b + o_err) + 10;     // [2], likewise
    c->w.lay_base = (int *)(b + o_lb);
    c->w.lay_mask = (uint64_t *)(b + o_lm);
    c->w.lay = (uint16_t *)(b + o_lay);
    c->w.deep = (int *)(b + o_deep);
    c->w.xlist = (int *)(b + o_xl);
    c->w.stamps = (unsigned long long *)(b + o_stamp);
    c->w.ovf = (int *)(b + o_ovf);
    c->w.meta = (dcr::RecMeta *)(b + o_meta);
    c->w.rmeta = (uint2 *)(b + o_rm);
    c->w.rows = (uint4 *)(b + o_rows);
    return DCR_OK;
}

int dcr_run_batch(dcr_ctx *c, const dcr_batch *in, dcr_out *ss, dcr_out *ds) {
    if (!c || !in || !ss || !ds) return fail(DCR_EARG, "NULL argument");
    if (in->n_fam < 0 || in->n_reads < 0) return fail(DCR_EARG, "negative batch size");
    int rc = dcr_reserve(c, in);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemsetAsync(c->w.err, 0, 64, c->stream));
    c->last_reads = in->n_reads;
    // per-read preprocessing (:191-325) is fused: k_recmeta<ss> analyses the
    // clips and fully preprocesses the reads of records the fast kernel does
    // not take; the fast kernel does the 3' trim of its own records
    HIP_TRY(hipEventRecord(c->ev[0], c->stream));
    dcr::Args a;
    a.in = *in;
    a.P = c->d_params;
    std::memcpy(&a.ws, &c->w, sizeof(a.ws));
    a.ss = *ss;
    a.ds = *ds;
    a.fast_ok = c->fast_ok;
    a.t16 = c->wide_ok ? c->fast_t16 : -1;     // -1: no decision pass
    a.wtab = c->d_wtab;
    // per strand: k_recmeta classifies every record (fast list / general list /
    // status written), then the fast kernel (8 records per wave) drains the fast list and
    // the persistent general kernel the rest (insertions, > 64 reads, wide layouts)
    auto grid_for = [&](int64_t n_rec, unsigned cap) {
        return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n_rec + 3) / 4, cap));
    };
    // persistent fast kernel: the resident blocks (16 waves each), at least
    // ~8 records per wave
    auto fast_grid = [&](int64_t n_rec, int k) {
        return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n_rec + 127) / 128, (int64_t)c->fast_blocks[k] * c->n_cu));
    };
    // k_fast_rows: one lane per fast-list entry (the list is at most n_rec long)
    auto rows_grid = [&](int64_t n_rec) { return (unsigned)std::max<int64_t>(1, (n_rec + 255) / 256); };
    auto fast_args = [&](bool duplex) {
        dcr::FastArgs f{};
        f.gb = duplex ? ss->seq : in->bases;
        f.gq = duplex ? ss->qual : in->quals;
        f.nbytes = duplex ? in->ss_cols : in->n_bases;
        f.meta = c->w.meta;
        f.rows = c->w.rows;
        f.rmeta = c->w.rmeta;
        f.fast_count = c->w.fast_count + (duplex ? 1 : 0);
        f.info = c->w.info;
        f.norm_cig = c->w.norm_cig;
        f.cig_off = in->cig_off;
        f.ovf = c->w.ovf;
        f.ovf_count = c->w.ovf_count + (duplex ? 1 : 0);
        f.xlist = c->w.xlist;
        f.xcount = c->w.xcount + (duplex ? 1 : 0);
        f.O = duplex ? *ds : *ss;
        f.P = c->d_params;
        f.stamps = c->w.stamps;
        f.kq = c->fast_kq;
        f.kqlo = c->fast_kqlo;
        f.maxq = c->fast_maxq;
        f.t16 = c->fast_t16;
        f.r_safe = c->fast_r_safe;
        f.minbq = duplex ? -1 : c->host_params.min_base_quality;
        f.lo_check = duplex || c->host_params.min_base_quality < c->fast_qlo;
        f.llr16 = c->d_llr16;
        f.llr8 = c->d_llr8;
        f.r2tab = c->d_r2tab;
        f.t8 = c->fast_t8;
        f.narrow = c->fast_narrow;
        f.e1000 = c->d_e1000;
        {
            // record-scalar stores at 32-bit offsets from the lowest array
            // (k_consensus_fast): every array + its largest index within 4 GiB
            const dcr_out &O = f.O;
            const int64_t nrec = (duplex ? 2 : 4) * in->n_fam, ncol = duplex ? in->ds_cols : in->ss_cols;
            const uint8_t *p[10] = {(const uint8_t *)O.pos, (const uint8_t *)O.mapq, (const uint8_t *)O.len,
                                    (const uint8_t *)O.n_cig, (const uint8_t *)O.n_de, (const uint8_t *)O.D,
                                    (const uint8_t *)O.M, (const uint8_t *)O.E, (const uint8_t *)O.E + 4,
                                    (const uint8_t *)O.cigar};
            const uint8_t *lo = p[0];
            for (int k = 1; k < 10; ++k) lo = std::min(lo, p[k]);
            bool ok = lo != nullptr;
            for (int k = 0; k < 10 && ok; ++k) {
                const uint64_t reach = (uint64_t)(p[k] - lo) + (k == 9 ? 4 * (uint64_t)ncol : (k == 7 || k == 8 ? 8 : 4) * (uint64_t)nrec);
                ok = p[k] != nullptr && reach < 0xFFFFFFF0ull;
                f.sofs[k] = (uint32_t)(p[k] - lo);
            }
            f.sbase = ok ? (uint8_t *)lo : nullptr;
        }
        f.want_info = (c->options & DCR_OPT_READ_INFO) ? 1 : 0;
        f.direct_r = duplex ? 0 : c->direct_r;
        return f;
    };
    auto strand = [&](bool duplex) -> int {
        a.n_rec = (duplex ? 2LL : 4LL) * in->n_fam;
        const dcr::FastArgs fa = fast_args(duplex);
        // k_recmeta: 64 records per wave, or fewer when the reads per record
        // exceed 16 on average (about 1,024 reads per wave)
        int rpw = 64;
        if (!duplex && a.n_rec > 0) {
            const int64_t avg = (int64_t)in->n_reads / a.n_rec;
            while (rpw > 1 && (int64_t)rpw * avg > 1024) rpw >>= 1;
        }
        a.rpw = rpw;
        const int rm_waves = rpw == 64 ? c->rm_waves : 4;           // heavy records: small blocks
        const int64_t rpb = (int64_t)rm_waves * rpw;                // records per k_recmeta block
        const unsigned nb = (unsigned)((a.n_rec + rpb - 1) / rpb);
        const size_t rm_lds = dcr::recmeta_lds_bytes(rm_waves);
        hipEvent_t *ev = c->ev + (duplex ? 5 : 1);
        // the exact queue is filled by the common kernel; its length is only
        // known on the device, so the exact kernel gets the resident grid
        const unsigned gx = (unsigned)((int64_t)c->fast_blocks[duplex ? 3 : 2] * c->n_cu);
        if (duplex) {
            hipLaunchKernelGGL(dcr::k_recmeta<true>, dim3(nb), dim3(rm_waves * dcr::kWave), rm_lds, c->stream, a);
            HIP_TRY(hipEventRecord(ev[0], c->stream));
            hipLaunchKernelGGL((dcr::k_consensus_fast<true, false>), dim3(fast_grid(a.n_rec, 1)), dim3(dcr::kFastBlock),
                               0, c->stream, fa);
            hipLaunchKernelGGL(dcr::k_fast_rows, dim3(rows_grid(a.n_rec)), dim3(256), 0, c->stream, fa);
            HIP_TRY(hipEventRecord(ev[1], c->stream));
            hipLaunchKernelGGL((dcr::k_consensus_fast<true, true>), dim3(gx), dim3(dcr::kFastBlock), 0, c->stream, fa);
            HIP_TRY(hipEventRecord(ev[2], c->stream));
            hipLaunchKernelGGL(dcr::k_decide<true>, dim3(grid_for(a.n_rec, 2048)), dim3(256), 0, c->stream, a);
            if (DCR_LAYOUT_KERNEL)
                hipLaunchKernelGGL(dcr::k_ins_layout<true>, dim3(grid_for(a.n_rec, 2048)), dim3(256), 0, c->stream, a);
            hipLaunchKernelGGL(dcr::k_consensus_general<true>, dim3(grid_for(a.n_rec, 1024)), dim3(256), 0,
                               c->stream, a);
        } else {
            hipLaunchKernelGGL(dcr::k_recmeta<false>, dim3(nb), dim3(rm_waves * dcr::kWave), rm_lds, c->stream, a);
            if (c->max_r_hint < 0 || c->max_r_hint > dcr::kWave)
                hipLaunchKernelGGL(dcr::k_prep_big, dim3(grid_for(a.n_rec, 2048)), dim3(256), 0, c->stream, a);
            HIP_TRY(hipEventRecord(ev[0], c->stream));
            hipLaunchKernelGGL((dcr::k_consensus_fast<false, false>), dim3(fast_grid(a.n_rec, 0)),
                               dim3(dcr::kFastBlock), 0, c->stream, fa);
            hipLaunchKernelGGL(dcr::k_fast_rows, dim3(rows_grid(a.n_rec)), dim3(256), 0, c->stream, fa);
            HIP_TRY(hipEventRecord(ev[1], c->stream));
            hipLaunchKernelGGL((dcr::k_consensus_fast<false, true>), dim3(gx), dim3(dcr::kFastBlock), 0, c->stream, fa);
            HIP_TRY(hipEventRecord(ev[2], c->stream));
            hipLaunchKernelGGL(dcr::k_decide<false>, dim3(grid_for(a.n_rec, 2048)), dim3(256), 0, c->stream, a);
            // (its 66 KB blocks wait for room beside the inflate waves in the
            // whole-node pipeline even when they find no deep record: up to
            // 7 ms per C2 pass, profiles/r06g)
            if (c->max_r_hint < 0 || c->max_r_hint >= dcr::kDeepReads)
                hipLaunchKernelGGL(dcr::k_decide_deep, dim3(2 * c->n_cu), dim3(dcr::kDeepWaves * dcr::kWave), 0, c->stream,
                                   a);
            // after k_decide_deep: it reads the general list's entries, which
            // k_ins_layout marks decided (bit 31) for the records it decides
            if (DCR_LAYOUT_KERNEL)
                hipLaunchKernelGGL(dcr::k_ins_layout<false>, dim3(grid_for(a.n_rec, 2048)), dim3(256), 0, c->stream, a);
            hipLaunchKernelGGL(dcr::k_consensus_general<false>, dim3(grid_for(a.n_rec, 1024)), dim3(256), 0,
                               c->stream, a);
        }
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(ev[3], c->stream));
        return DCR_OK;
    };
    if (in->n_fam > 0) {
        if ((rc = strand(false))) return rc;
        if ((rc = strand(true))) return rc;
    } else {
        for (int k = 1; k <= DCR_N_KERNEL_TIMES; ++k) HIP_TRY(hipEventRecord(c->ev[k], c->stream));
    }
    c->timed = true;
    return DCR_OK;
}

int dcr_sync(dcr_ctx *c) {
    if (!c) return fail(DCR_EARG, "ctx is NULL");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->w.err) {
        int err = 0;
        HIP_TRY(hipMemcpy(&err, c->w.err, sizeof(int), hipMemcpyDeviceToHost));
        if (err) return fail(DCR_ECAPACITY, "a consensus needed more columns than its output region");
    }
    return DCR_OK;
}

int dcr_last_timing(dcr_ctx *c, float *ms4) {
    if (!c || !ms4) return fail(DCR_EARG, "NULL argument");
    if (!c->timed) return fail(DCR_EARG, "no batch has run");
    const int last = DCR_N_KERNEL_TIMES;
    HIP_TRY(hipEventSynchronize(c->ev[last]));
    ms4[0] = 0.0f;                       // preprocessing is fused into k_recmeta / the fast kernel
    HIP_TRY(hipEventElapsedTime(&ms4[1], c->ev[0], c->ev[4]));
    HIP_TRY(hipEventElapsedTime(&ms4[2], c->ev[4], c->ev[last]));
    HIP_TRY(hipEventElapsedTime(&ms4[3], c->ev[0], c->ev[last]));
    return DCR_OK;
}

// diagnostic (not in include/dcr.h): phase cycle counters of DCR_STAMP builds
int dcr_debug_stamps(dcr_ctx *c, unsigned long long *out, int n, int reset) {
    if (!c || !out || n > 64) return fail(DCR_EARG, "bad argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipMemcpy(out, c->w.stamps, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost));
    if (reset) HIP_TRY(hipMemset(c->w.stamps, 0, sizeof(unsigned long long) * 64));
    return DCR_OK;
}

// diagnostic (not in include/dcr.h): the last batch's queue counters -- err,
// ovf_count[2], fast_count[2], xcount[2] (exact queue), gen_next[2], deep_count
int dcr_debug_counts(dcr_ctx *c, int *out10) {
    if (!c || !out10) return fail(DCR_EARG, "NULL argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipMemcpy(out10, c->w.err, sizeof(int) * 10, hipMemcpyDeviceToHost));
    return DCR_OK;
}

int dcr_last_kernel_timing(dcr_ctx *c, float *ms) {
    if (!c || !ms) return fail(DCR_EARG, "NULL argument");
    if (!c->timed) return fail(DCR_EARG, "no batch has run");
    HIP_TRY(hipEventSynchronize(c->ev[DCR_N_KERNEL_TIMES]));
    for (int k = 0; k < DCR_N_KERNEL_TIMES; ++k) HIP_TRY(hipEventElapsedTime(&ms[k], c->ev[k], c->ev[k + 1]));
    return DCR_OK;
}

int dcr_read_info_host(dcr_ctx *c, dcr_read_info *out, int64_t n) {
    if (!c || !out) return fail(DCR_EARG, "NULL argument");
    if (n > c->last_reads) return fail(DCR_EARG, "more reads requested than the last batch held");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (n > 0) HIP_TRY(hipMemcpy(out, c->w.info, sizeof(dcr_read_info) * n, hipMemcpyDeviceToHost));
    return DCR_OK;
}

// Device layout of one batch's inputs and outputs in a single buffer:
// returns the bytes needed; with base != nullptr also fills the device
// views db (inputs) and dout[0..1] (single-strand, duplex outputs).
static size_t plan_io(const dcr_batch *h, char *base, dcr_batch *db, dcr_out dout[2]) {
    const int64_t F = h->n_fam, n = h->n_reads;
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off = align_up(off + std::max<size_t>(bytes, 1)); return o; };
    const size_t o_sub = take(sizeof(int32_t) * (4 * F + 1));
    const size_t o_pos = take(sizeof(int32_t) * n);
    const size_t o_mq = take(n);
    const size_t o_so = take(sizeof(int64_t) * n);
    const size_t o_sl = take(sizeof(int32_t) * n);
    const size_t o_co = take(sizeof(int32_t) * n);
    const size_t o_cn = take(sizeof(int32_t) * n);
    const size_t o_cg = take(sizeof(uint32_t) * h->n_cigar);
    const size_t o_b = take(h->n_bases);
    const size_t o_q = take(h->n_bases);
    const size_t o_sc = take(sizeof(int64_t) * (4 * F + 1));
    const size_t o_dc = take(sizeof(int64_t) * (2 * F + 1));
    size_t oo[2][14];
    const int64_t nrec[2] = {4 * F, 2 * F};
    const int64_t ncol[2] = {h->ss_cols, h->ds_cols};
    for (int k = 0; k < 2; ++k) {
        oo[k][0] = take(nrec[k]);
        for (int j = 1; j <= 7; ++j) oo[k][j] = take(sizeof(int32_t) * nrec[k]);
        oo[k][8] = take(sizeof(double) * nrec[k]);
        oo[k][9] = take(ncol[k]);
        oo[k][10] = take(ncol[k]);
        oo[k][11] = take(sizeof(uint32_t) * ncol[k]);
        oo[k][12] = take(sizeof(uint16_t) * ncol[k]);
        oo[k][13] = take(sizeof(uint16_t) * ncol[k]);
    }
    if (!base) return off;
    char *d = base;
    *db = *h;
    db->sub_off = (const int32_t *)(d + o_sub);
    db->read_pos = (const int32_t *)(d + o_pos);
    db->read_mapq = (const uint8_t *)(d + o_mq);
    db->seq_off = (const int64_t *)(d + o_so);
    db->seq_len = (const int32_t *)(d + o_sl);
    db->cig_off = (const int32_t *)(d + o_co);
    db->cig_n = (const int32_t *)(d + o_cn);
    db->cigar = (const uint32_t *)(d + o_cg);
    db->bases = (const uint8_t *)(d + o_b);
    db->quals = (const uint8_t *)(d + o_q);
    db->ss_col_off = (const int64_t *)(d + o_sc);
    db->ds_col_off = (const int64_t *)(d + o_dc);
    for (int k = 0; k < 2; ++k) {
        dout[k].status = (uint8_t *)(d + oo[k][0]);
        dout[k].pos = (int32_t *)(d + oo[k][1]);
        dout[k].mapq = (int32_t *)(d + oo[k][2]);
        dout[k].len = (int32_t *)(d + oo[k][3]);
        dout[k].n_cig = (int32_t *)(d + oo[k][4]);
        dout[k].n_de = (int32_t *)(d + oo[k][5]);
        dout[k].D = (int32_t *)(d + oo[k][6]);
        dout[k].M = (int32_t *)(d + oo[k][7]);
        dout[k].E = (double *)(d + oo[k][8]);
        dout[k].seq = (uint8_t *)(d + oo[k][9]);
        dout[k].qual = (uint8_t *)(d + oo[k][10]);
        dout[k].cigar = (uint32_t *)(d + oo[k][11]);
        dout[k].d = (uint16_t *)(d + oo[k][12]);
        dout[k].e = (uint16_t *)(d + oo[k][13]);
    }
    return off;
}

// the host batch's inputs -> device views (async on stream s)
static hipError_t upload_inputs(const dcr_batch *h, const dcr_batch &db, hipStream_t s) {
    const int64_t F = h->n_fam, n = h->n_reads;
    struct P { void *dst; const void *src; size_t bytes; } ps[12] = {
        {(void *)db.sub_off, h->sub_off, sizeof(int32_t) * (4 * F + 1)},
        {(void *)db.read_pos, h->read_pos, sizeof(int32_t) * n},
        {(void *)db.read_mapq, h->read_mapq, (size_t)n},
        {(void *)db.seq_off, h->seq_off, sizeof(int64_t) * n},
        {(void *)db.seq_len, h->seq_len, sizeof(int32_t) * n},
        {(void *)db.cig_off, h->cig_off, sizeof(int32_t) * n},
        {(void *)db.cig_n, h->cig_n, sizeof(int32_t) * n},
        {(void *)db.cigar, h->cigar, sizeof(uint32_t) * h->n_cigar},
        {(void *)db.bases, h->bases, (size_t)h->n_bases},
        {(void *)db.quals, h->quals, (size_t)h->n_bases},
        {(void *)db.ss_col_off, h->ss_col_off, sizeof(int64_t) * (4 * F + 1)},
        {(void *)db.ds_col_off, h->ds_col_off, sizeof(int64_t) * (2 * F + 1)}};
    for (auto &p : ps)
        if (p.bytes) {
            hipError_t e = hipMemcpyAsync(p.dst, p.src, p.bytes, hipMemcpyHostToDevice, s);
            if (e != hipSuccess) return e;
        }
    return hipSuccess;
}

// device outputs -> the host dcr_out arrays that are not NULL (async on stream s)
static hipError_t download_outputs(const dcr_out *dev, dcr_out *host, int64_t R, int64_t C, hipStream_t s) {
    struct P { void *dst; const void *src; size_t bytes; } ps[14] = {
        {host->status, dev->status, (size_t)R}, {host->pos, dev->pos, 4 * (size_t)R},
        {host->mapq, dev->mapq, 4 * (size_t)R}, {host->len, dev->len, 4 * (size_t)R},
        {host->n_cig, dev->n_cig, 4 * (size_t)R}, {host->n_de, dev->n_de, 4 * (size_t)R},
        {host->D, dev->D, 4 * (size_t)R}, {host->M, dev->M, 4 * (size_t)R}, {host->E, dev->E, 8 * (size_t)R},
        {host->seq, dev->seq, (size_t)C}, {host->qual, dev->qual, (size_t)C},
        {host->cigar, dev->cigar, 4 * (size_t)C}, {host->d, dev->d, 2 * (size_t)C}, {host->e, dev->e, 2 * (size_t)C}};
    for (auto &p : ps)
        if (p.dst && p.bytes) {
            hipError_t e = hipMemcpyAsync(p.dst, p.src, p.bytes, hipMemcpyDeviceToHost, s);
            if (e != hipSuccess) return e;
        }
    return hipSuccess;
}

// host-pointer entry point: one staging allocation, H2D, run, D2H
int dcr_run_batch_host(dcr_ctx *c, const dcr_batch *h, dcr_out *hss, dcr_out *hds) {
    if (!c || !h || !hss || !hds) return fail(DCR_EARG, "NULL argument");
    HIP_TRY(hipSetDevice(c->device));
    const size_t need = plan_io(h, nullptr, nullptr, nullptr);
    if (need > c->io.cap) {
        HIP_TRY(hipStreamSynchronize(c->stream));
        HIP_TRY(c->io.ensure(need));
    }
    dcr_batch db;
    dcr_out dout[2];
    plan_io(h, (char *)c->io.p, &db, dout);
    HIP_TRY(upload_inputs(h, db, c->stream));
    int rc = dcr_run_batch(c, &db, &dout[0], &dout[1]);
    if (rc) return rc;
    HIP_TRY(download_outputs(&dout[0], hss, 4 * (int64_t)h->n_fam, h->ss_cols, c->stream));
    HIP_TRY(download_outputs(&dout[1], hds, 2 * (int64_t)h->n_fam, h->ds_cols, c->stream));
    return dcr_sync(c);
}

// ---- streaming (pinned host batches, per-slot device buffers, copy streams) ----

void *dcr_host_alloc(size_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 16, hipHostMallocDefault) != hipSuccess) {
        g_err = "hipHostMalloc failed";
        return nullptr;
    }
    return p;
}

void dcr_host_free(void *p) {
    if (p) (void)hipHostFree(p);
}

// the largest subfamily of a host batch (sub_off is a host array here)
static int host_max_r(const dcr_batch *h) {
    int m = 0;
    const int64_t n = 4 * (int64_t)h->n_fam;
    if (n > 0 && !h->sub_off) return -1;
    for (int64_t i = 0; i < n; ++i) m = std::max(m, h->sub_off[i + 1] - h->sub_off[i]);
    return m;
}

int dcr_submit(dcr_ctx *c, int slot, const dcr_batch *h, dcr_out *hss, dcr_out *hds, int32_t *read_status) {
    if (!c || !h || !hss || !hds) return fail(DCR_EARG, "NULL argument");
    if (slot < 0 || slot >= DCR_MAX_SLOTS) return fail(DCR_EARG, "slot out of range");
    HIP_TRY(hipSetDevice(c->device));
    if (!c->s_h2d) {
        HIP_TRY(hi_prio_stream(&c->s_h2d));
        HIP_TRY(hi_prio_stream(&c->s_d2h));
        HIP_TRY(hi_prio_stream(&c->s_fetch));
    }
    dcr_ctx::Slot &S = c->slots[slot];
    if (!S.ev_h2d) {
        HIP_TRY(hipEventCreateWithFlags(&S.ev_h2d, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&S.ev_comp, hipEventDisableTiming));
        // the host waits on this one (dcr_wait / dcr_wait_write): blocking, so the
        // waiting thread sleeps instead of spinning on a core the ingest needs
        HIP_TRY(hipEventCreateWithFlags(&S.ev_d2h, hipEventDisableTiming | hipEventBlockingSync));
        HIP_TRY(hipHostMalloc((void **)&S.h_err, sizeof(int), hipHostMallocDefault));
        *S.h_err = 0;
    }
    if (S.busy) return fail(DCR_EARG, "slot still in flight (dcr_wait it first)");
    const size_t need = plan_io(h, nullptr, nullptr, nullptr);
    if (need > S.buf.cap) HIP_TRY(S.buf.ensure(need + need / 8));   // idle slot: nothing in flight uses it
    dcr_batch db;
    dcr_out dout[2];
    plan_io(h, (char *)S.buf.p, &db, dout);
    // H2D on the copy stream
    HIP_TRY(upload_inputs(h, db, c->s_h2d));
    HIP_TRY(hipEventRecord(S.ev_h2d, c->s_h2d));
    // kernels on the compute stream
    HIP_TRY(hipStreamWaitEvent(c->stream, S.ev_h2d, 0));
    c->max_r_hint = host_max_r(h);
    int rc = dcr_run_batch(c, &db, &dout[0], &dout[1]);
    c->max_r_hint = -1;
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(S.h_err, c->w.err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    if (read_status && h->n_reads > 0)
        HIP_TRY(hipMemcpy2DAsync(read_status, sizeof(int32_t), (const char *)c->w.info + offsetof(dcr_read_info, status),
                                 sizeof(dcr_read_info), sizeof(int32_t), (size_t)h->n_reads, hipMemcpyDeviceToHost,
                                 c->stream));
    HIP_TRY(hipEventRecord(S.ev_comp, c->stream));
    // D2H of the outputs on the second copy stream
    HIP_TRY(hipStreamWaitEvent(c->s_d2h, S.ev_comp, 0));
    HIP_TRY(download_outputs(&dout[0], hss, 4 * (int64_t)h->n_fam, h->ss_cols, c->s_d2h));
    HIP_TRY(download_outputs(&dout[1], hds, 2 * (int64_t)h->n_fam, h->ds_cols, c->s_d2h));
    HIP_TRY(hipEventRecord(S.ev_d2h, c->s_d2h));
    S.writer = false;
    S.busy = true;
    return DCR_OK;
}

int dcr_wait(dcr_ctx *c, int slot) {
    if (!c || slot < 0 || slot >= DCR_MAX_SLOTS) return fail(DCR_EARG, "bad argument");
    dcr_ctx::Slot &S = c->slots[slot];
    if (!S.busy) return DCR_OK;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipEventSynchronize(S.ev_d2h));
    S.busy = false;
    if (*S.h_err) return fail(DCR_ECAPACITY, "a consensus needed more columns than its output region");
    return DCR_OK;
}


// ---- device record writer ----------------------------------------------------

// Upper bound of the formatted duplex records of a batch (dcr_writer.hip
// rec_size): regions bound lengths, CIGARs and depth lists.
static int64_t stream_bound(const dcr_batch *h, const dcr_wmeta *m) {
    int64_t B = 0;
    for (int32_t f = 0; f < h->n_fam; ++f) {
        const int64_t lc = (int64_t)std::strlen(m->names + m->fam_code[f]);
        for (int j = 0; j < 2; ++j) {
            const int a = 4 * f + 2 * j, b = a + 1;
            const int64_t Td = h->ds_col_off[2 * f + j + 1] - h->ds_col_off[2 * f + j];
            const int64_t Ta = h->ss_col_off[a + 1] - h->ss_col_off[a];
            const int64_t Tb = h->ss_col_off[b + 1] - h->ss_col_off[b];
            const int64_t lr = (int64_t)std::strlen(m->names + m->fam_rx[2 * f + j]);
            B += 400 + 2 * lc + lr + 20 * Td + 16 * (Ta + Tb) + (h->sub_off[a + 1] - h->sub_off[a]) +
                 (h->sub_off[b + 1] - h->sub_off[b]);
        }
    }
    return B;
}

int dcr_submit_write(dcr_ctx *c, int slot, const dcr_batch *h, const dcr_wmeta *m, dcr_wres *res) {
    if (!c || !h || !m || !res) return fail(DCR_EARG, "NULL argument");
    if (slot < 0 || slot >= DCR_MAX_SLOTS) return fail(DCR_EARG, "slot out of range");
    HIP_TRY(hipSetDevice(c->device));
    if (!c->s_h2d) {
        HIP_TRY(hi_prio_stream(&c->s_h2d));
        HIP_TRY(hi_prio_stream(&c->s_d2h));
        HIP_TRY(hi_prio_stream(&c->s_fetch));
    }
    dcr_ctx::Slot &S = c->slots[slot];
    if (!S.ev_h2d) {
        HIP_TRY(hipEventCreateWithFlags(&S.ev_h2d, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&S.ev_comp, hipEventDisableTiming));
        // the host waits on this one (dcr_wait / dcr_wait_write): blocking, so the
        // waiting thread sleeps instead of spinning on a core the ingest needs
        HIP_TRY(hipEventCreateWithFlags(&S.ev_d2h, hipEventDisableTiming | hipEventBlockingSync));
        HIP_TRY(hipHostMalloc((void **)&S.h_err, sizeof(int), hipHostMallocDefault));
        *S.h_err = 0;
    }
    if (S.busy) return fail(DCR_EARG, "slot still in flight (dcr_wait it first)");
    const int64_t F = h->n_fam;
    // consensus buffers
    const size_t need = plan_io(h, nullptr, nullptr, nullptr);
    if (need > S.buf.cap) HIP_TRY(S.buf.ensure(need + need / 8));
    dcr_batch db;
    dcr_out dout[2];
    plan_io(h, (char *)S.buf.p, &db, dout);
    // writer buffers
    const int64_t B = stream_bound(h, m);
    const int64_t nbm = B / (int64_t)dfl::kMaxIn + 2;
    const size_t scan1 = dcrw::scan_tmp_bytes((int)(2 * F + 1)), scan2 = dcrw::scan_tmp_bytes((int)(nbm + 1));
    size_t wo = 0;
    auto take = [&](size_t bytes) { size_t o = wo; wo = align_up(wo + std::max<size_t>(bytes, 1)); return o; };
    const size_t o_names = take((size_t)m->n_names + 1);
    const size_t o_code = take(8 * (size_t)F), o_rx = take(16 * (size_t)F), o_tid = take(4 * (size_t)F);
    const size_t o_fail = take(4 * (size_t)F), o_dlen = take(8 * (size_t)F);
    const size_t o_rsz = take(8 * (size_t)(2 * F + 1)), o_roff = take(8 * (size_t)(2 * F + 1));
    const size_t o_scan = take(std::max(scan1, scan2));
    const size_t o_stream = take((size_t)B);
    const size_t o_slots = take((size_t)nbm * dfl::kSlot);
    // block sizes (+ the scan's total), then k_deflate's block counter
    const size_t o_bsz = take(8 * (size_t)(nbm + 2)), o_boff = take(8 * (size_t)(nbm + 1));
    const size_t o_comp = take((size_t)nbm * dfl::kSlot);
    const size_t o_tot = take(8 * 4);
    const unsigned gd = (unsigned)std::max<int64_t>(1, std::min<int64_t>(nbm, (int64_t)c->n_cu * c->dfl_blocks));
    const size_t o_tok = take((size_t)gd * dfl::kTokWords * 4);
    if (wo > S.wbuf.cap) HIP_TRY(S.wbuf.ensure(wo + wo / 8));
    char *wb = (char *)S.wbuf.p;
    // H2D: inputs and writer metadata on the copy stream
    HIP_TRY(upload_inputs(h, db, c->s_h2d));
    if (m->n_names) HIP_TRY(hipMemcpyAsync(wb + o_names, m->names, (size_t)m->n_names, hipMemcpyHostToDevice, c->s_h2d));
    if (F) {
        HIP_TRY(hipMemcpyAsync(wb + o_code, m->fam_code, 8 * (size_t)F, hipMemcpyHostToDevice, c->s_h2d));
        HIP_TRY(hipMemcpyAsync(wb + o_rx, m->fam_rx, 16 * (size_t)F, hipMemcpyHostToDevice, c->s_h2d));
        HIP_TRY(hipMemcpyAsync(wb + o_tid, m->fam_tid, 4 * (size_t)F, hipMemcpyHostToDevice, c->s_h2d));
    }
    HIP_TRY(hipEventRecord(S.ev_h2d, c->s_h2d));
    // consensus kernels on the compute stream
    HIP_TRY(hipStreamWaitEvent(c->stream, S.ev_h2d, 0));
    c->max_r_hint = host_max_r(h);
    int rc = dcr_run_batch(c, &db, &dout[0], &dout[1]);
    c->max_r_hint = -1;
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(S.h_err, c->w.err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    // record writer
    dcrw::FmtArgs A{};
    A.ss = dout[0];
    A.ds = dout[1];
    A.sub_off = db.sub_off;
    A.read_mapq = db.read_mapq;
    A.ss_col_off = db.ss_col_off;
    A.ds_col_off = db.ds_col_off;
    A.info = c->w.info;
    A.names = wb + o_names;
    A.fam_code = (const int64_t *)(wb + o_code);
    A.fam_rx = (const int64_t *)(wb + o_rx);
    A.fam_tid = (const int32_t *)(wb + o_tid);
    A.n_fam = (int32_t)F;
    A.fam_fail = (int32_t *)(wb + o_fail);
    A.ds_len_out = (int32_t *)(wb + o_dlen);
    int64_t *rsz = (int64_t *)(wb + o_rsz);
    A.rec_size = rsz;
    A.rec_off = (int64_t *)(wb + o_roff);
    A.stream = (uint8_t *)(wb + o_stream);
    HIP_TRY(hipMemsetAsync(rsz, 0, 8 * (size_t)(2 * F + 1), c->stream));
    HIP_TRY(hipMemsetAsync(wb + o_bsz, 0, 8 * (size_t)(nbm + 2), c->stream));
    if (F) {
        hipLaunchKernelGGL(dcrw::k_famfail, dim3((unsigned)((F + 255) / 256)), dim3(256), 0, c->stream, A);
        const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((2 * F + 3) / 4, (int64_t)c->n_cu * 8));
        hipLaunchKernelGGL(dcrw::k_fmt_size, dim3(g), dim3(256), 0, c->stream, A);
        HIP_TRY(hipGetLastError());
        HIP_TRY(dcrw::scan_excl_i64(rsz, A.rec_off, (int)(2 * F + 1), (int64_t *)(wb + o_scan), c->stream));
        hipLaunchKernelGGL(dcrw::k_fmt_write, dim3(g), dim3(256), 0, c->stream, A);
        HIP_TRY(hipGetLastError());
    } else {
        HIP_TRY(hipMemsetAsync(A.rec_off, 0, 8, c->stream));
    }
    int64_t *bsz = (int64_t *)(wb + o_bsz);
    dcrw::DflArgs D{A.stream, A.rec_off + 2 * F, (uint8_t *)(wb + o_slots), bsz, (uint32_t *)(wb + o_tok), nullptr,
                    DFL_CLAIM ? (unsigned long long *)(bsz + nbm + 1) : nullptr};
    hipLaunchKernelGGL(dcrw::k_deflate, dim3(gd), dim3(dfl::kT), sizeof(dfl::Shared), c->stream, D);
    HIP_TRY(hipGetLastError());
    int64_t *boff = (int64_t *)(wb + o_boff);
    HIP_TRY(dcrw::scan_excl_i64(bsz, boff, (int)(nbm + 1), (int64_t *)(wb + o_scan), c->stream));
    dcrw::CompactArgs C{(const uint8_t *)(wb + o_slots), bsz, boff, A.rec_off + 2 * F,
                        (uint8_t *)(wb + o_comp), (int64_t *)(wb + o_tot)};
    hipLaunchKernelGGL(dcrw::k_compact, dim3(gd), dim3(256), 0, c->stream, C);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(S.ev_comp, c->stream));
    // D2H of the per-family outcome and the totals on the second copy stream
    HIP_TRY(hipStreamWaitEvent(c->s_d2h, S.ev_comp, 0));
    if (F) {
        HIP_TRY(hipMemcpyAsync(res->fam_fail, A.fam_fail, 4 * (size_t)F, hipMemcpyDeviceToHost, c->s_d2h));
        HIP_TRY(hipMemcpyAsync(res->ds_len, A.ds_len_out, 8 * (size_t)F, hipMemcpyDeviceToHost, c->s_d2h));
    }
    HIP_TRY(hipMemcpyAsync(res->totals, wb + o_tot, 3 * sizeof(int64_t), hipMemcpyDeviceToHost, c->s_d2h));
    HIP_TRY(hipEventRecord(S.ev_d2h, c->s_d2h));
    S.d_rec_off = A.rec_off;
    S.d_stream = A.stream;
    S.d_comp = (uint8_t *)(wb + o_comp);
    S.n_fam = F;
    S.writer = true;
    S.busy = true;
    return DCR_OK;
}

int dcr_wait_write(dcr_ctx *c, int slot, dcr_wres *res) {
    if (!c || !res || slot < 0 || slot >= DCR_MAX_SLOTS) return fail(DCR_EARG, "bad argument");
    dcr_ctx::Slot &S = c->slots[slot];
    if (!S.busy || !S.writer) return fail(DCR_EARG, "slot has no writer batch in flight");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipEventSynchronize(S.ev_d2h));
    S.busy = false;
    if (*S.h_err) return fail(DCR_ECAPACITY, "a consensus needed more columns than its output region");
    const int64_t n = res->totals[0];
    if (n > res->cap_bgzf) return fail(DCR_ECAPACITY, "BGZF output larger than cap_bgzf (see totals[0])");
    if (n > 0) {
        if (!c->ev_fetch) HIP_TRY(hipEventCreateWithFlags(&c->ev_fetch, hipEventDisableTiming | hipEventBlockingSync));
        HIP_TRY(hipMemcpyAsync(res->bgzf, S.d_comp, (size_t)n, hipMemcpyDeviceToHost, c->s_fetch));
        HIP_TRY(hipEventRecord(c->ev_fetch, c->s_fetch));
        HIP_TRY(hipEventSynchronize(c->ev_fetch));
    }
    return DCR_OK;
}

int dcr_slot_fetch(dcr_ctx *c, int slot, int what, int64_t off, int64_t n, void *dst) {
    if (!c || !dst || slot < 0 || slot >= DCR_MAX_SLOTS || off < 0 || n < 0) return fail(DCR_EARG, "bad argument");
    dcr_ctx::Slot &S = c->slots[slot];
    if (!S.writer) return fail(DCR_EARG, "slot holds no writer batch");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipEventSynchronize(S.ev_d2h));
    if (what == 0) {
        if (n) HIP_TRY(hipMemcpy(dst, S.d_stream + off, (size_t)n, hipMemcpyDeviceToHost));
    } else if (what == 1) {
        if (off + n > 2 * S.n_fam + 1) return fail(DCR_EARG, "record offsets out of range");
        if (n) HIP_TRY(hipMemcpy(dst, S.d_rec_off + off, 8 * (size_t)n, hipMemcpyDeviceToHost));
    } else if (what == 2) {
        if (n) HIP_TRY(hipMemcpy(dst, S.d_comp + off, (size_t)n, hipMemcpyDeviceToHost));
    } else {
        return fail(DCR_EARG, "what must be 0 (record bytes), 1 (record offsets) or 2 (BGZF blocks)");
    }
    return DCR_OK;
}

// diagnostic (not in include/dcr.h): k_deflate alone over n host bytes with
// per-phase s_memtime cycle totals (summed over workgroups) and the HIP-event
// time; returns the compressed bytes in *comp_bytes and, when slots_out is
// given (ceil(n / 0xff00) * 65536 bytes), each block's BGZF member at the
// start of its 64 KiB slot, the member sizes in sizes_out
int dcr_deflate_probe(dcr_ctx *c, const uint8_t *host, int64_t n, unsigned long long *stamps12, float *ms,
                      int64_t *comp_bytes, uint8_t *slots_out, int64_t *sizes_out) {
    if (!c || !host || n <= 0 || !stamps12 || !ms || !comp_bytes) return fail(DCR_EARG, "bad argument");
    HIP_TRY(hipSetDevice(c->device));
    const int64_t nb = (n + dfl::kMaxIn - 1) / dfl::kMaxIn;
    uint8_t *d_in = nullptr, *d_slots = nullptr;
    int64_t *d_n = nullptr, *d_sizes = nullptr;
    unsigned long long *d_st = nullptr;
    uint32_t *d_tok = nullptr;
    HIP_TRY(hipMalloc(&d_in, (size_t)n));
    HIP_TRY(hipMalloc(&d_slots, (size_t)nb * dfl::kSlot));
    HIP_TRY(hipMalloc(&d_n, 8));
    HIP_TRY(hipMalloc(&d_sizes, 8 * (size_t)nb));
    HIP_TRY(hipMalloc(&d_st, 8 * 12));
    const unsigned gd = (unsigned)std::max<int64_t>(1, std::min<int64_t>(nb, (int64_t)c->n_cu * c->dfl_blocks));
    HIP_TRY(hipMalloc(&d_tok, (size_t)gd * dfl::kTokWords * 4));
    HIP_TRY(hipMemcpy(d_in, host, (size_t)n, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(d_n, &n, 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemset(d_st, 0, 96));
    dcrw::DflArgs D{d_in, d_n, d_slots, d_sizes, d_tok, d_st, nullptr};
    hipEvent_t e0, e1;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, c->stream));
    hipLaunchKernelGGL(dcrw::k_deflate, dim3(gd), dim3(dfl::kT), sizeof(dfl::Shared), c->stream, D);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(e1, c->stream));
    HIP_TRY(hipEventSynchronize(e1));
    HIP_TRY(hipEventElapsedTime(ms, e0, e1));
    HIP_TRY(hipMemcpy(stamps12, d_st, 96, hipMemcpyDeviceToHost));
    std::vector<int64_t> sz((size_t)nb);
    HIP_TRY(hipMemcpy(sz.data(), d_sizes, 8 * (size_t)nb, hipMemcpyDeviceToHost));
    int64_t tot = 0;
    for (int64_t v : sz) tot += v;
    *comp_bytes = tot;
    if (sizes_out) std::memcpy(sizes_out, sz.data(), 8 * (size_t)nb);
    if (slots_out) HIP_TRY(hipMemcpy(slots_out, d_slots, (size_t)nb * dfl::kSlot, hipMemcpyDeviceToHost));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(d_in);
    (void)hipFree(d_slots);
    (void)hipFree(d_n);
    (void)hipFree(d_sizes);
    (void)hipFree(d_st);
    (void)hipFree(d_tok);
    return DCR_OK;
}

}  // extern "C"
