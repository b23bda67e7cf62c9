// libkwmatch multi-GPU exchange: RCCL over xGMI, one process per GPU.
//
// Matching shards with no data-path exchange (every article is independent,
// SURVEY.md §8(e)); the only collectives are the exchange of per-rank hit
// counts and of the packed 16-byte hit records, so that the rank that writes
// the output (or every rank) holds the records of the whole batch in document
// order.  This replaces the reference's process pool + shared filesystem
// (match_keywords.py:230-238: np.array_split + Pool.starmap), whose only
// "exchange" is the per-ticker CSV files every worker appends to.
//
// RCCL is resolved at run time (dlopen): the copy torch has already loaded
// (RTLD_NOLOAD, soname librccl.so.1) is reused so one process never holds two
// RCCL runtimes; otherwise /opt/rocm's.  Without RCCL the kw_comm_* calls fail
// with KW_EUNSUPPORTED; the single-GPU path never needs it.
#include <hip/hip_runtime.h>
#include <dlfcn.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/kwmatch.h"

namespace {

// the subset of rccl.h this file calls (types are ABI-stable in NCCL 2.x)
typedef struct ncclComm *ncclComm_t;
typedef struct { char internal[128]; } ncclUniqueId;
typedef int ncclResult_t;
enum { nccl_int8 = 0, nccl_uint32 = 3, nccl_int64 = 4 };

struct Rccl {
    void *so = nullptr;
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*AllGather)(const void *, void *, size_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Send)(const void *, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void *, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;
};

Rccl g_rccl;
std::string g_comm_err;

bool load_rccl(std::string &err)
{
    if (g_rccl.so) return true;
    void *so = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!so) so = dlopen("librccl.so.1", RTLD_NOW);
    if (!so) so = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
    if (!so) {
        err = std::string("kw_comm: RCCL (librccl.so.1) not found: ") + dlerror();
        return false;
    }
    Rccl r;
    r.so = so;
#define KW_SYM(field, name)                                                   \
    do {                                                                      \
        *(void **)(&r.field) = dlsym(so, name);                               \
        if (!r.field) { err = "kw_comm: RCCL symbol missing: " name; return false; } \
    } while (0)
    KW_SYM(GetUniqueId, "ncclGetUniqueId");
    KW_SYM(CommInitRank, "ncclCommInitRank");
    KW_SYM(CommDestroy, "ncclCommDestroy");
    KW_SYM(AllGather, "ncclAllGather");
    KW_SYM(Send, "ncclSend");
    KW_SYM(Recv, "ncclRecv");
    KW_SYM(GroupStart, "ncclGroupStart");
    KW_SYM(GroupEnd, "ncclGroupEnd");
    KW_SYM(GetErrorString, "ncclGetErrorString");
#undef KW_SYM
    g_rccl = r;
    return true;
}

// records of one rank -> global document ids (doc + base)
__global__ void kw_rebase_kernel(const kw_hit *__restrict__ src, kw_hit *__restrict__ dst, int64_t n, uint32_t base)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        kw_hit r = src[i];
        r.doc += base;
        dst[i] = r;
    }
}

}  // namespace

struct kw_comm {
    int nranks = 1, rank = 0, device = 0;
    ncclComm_t comm = nullptr;
    int64_t *d_counts = nullptr;   // [3 nranks + 3]: own values at [3 nranks, 3 nranks + 3), gathered at [0, 3 nranks)
    kw_hit *d_stage = nullptr;     // this rank's records, rebased
    size_t stage_cap = 0;
    kw_hit *d_spill = nullptr;     // a receiver's records when its destination is short (planned exchange)
    size_t spill_cap = 0;
    std::string err;
};

#define CCHK(c, x)                                                                          \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) { (c)->err = std::string("HIP error ") + hipGetErrorString(e_) + " at " #x; return KW_EHIP; } \
    } while (0)
#define NCHK(c, x)                                                                          \
    do {                                                                                    \
        ncclResult_t r_ = (x);                                                              \
        if (r_ != 0) { (c)->err = std::string("RCCL error: ") + g_rccl.GetErrorString(r_) + " at " #x; return KW_EHIP; } \
    } while (0)

extern "C" int kw_comm_unique_id(uint8_t *id_out)
{
    if (!id_out) return KW_EINVAL;
    if (!load_rccl(g_comm_err)) return KW_EUNSUPPORTED;
    ncclUniqueId id;
    ncclResult_t r = g_rccl.GetUniqueId(&id);
    if (r != 0) { g_comm_err = std::string("ncclGetUniqueId: ") + g_rccl.GetErrorString(r); return KW_EHIP; }
    memcpy(id_out, id.internal, KW_COMM_ID_BYTES);
    return KW_OK;
}

extern "C" int kw_comm_init(int32_t nranks, int32_t rank, const uint8_t *id, int32_t device, kw_comm **out)
{
    if (!out) return KW_EINVAL;
    *out = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks || !id) { g_comm_err = "kw_comm_init: bad arguments"; return KW_EINVAL; }
    if (!load_rccl(g_comm_err)) return KW_EUNSUPPORTED;
    kw_comm *c = new kw_comm();
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    *out = c;   // the caller reads kw_comm_last_error and destroys it on failure
    CCHK(c, hipSetDevice(device));
    ncclUniqueId uid;
    memcpy(uid.internal, id, KW_COMM_ID_BYTES);
    NCHK(c, g_rccl.CommInitRank(&c->comm, nranks, uid, rank));
    CCHK(c, hipMalloc(&c->d_counts, sizeof(int64_t) * (3 * nranks + 3)));
    return KW_OK;
}

// all-gather k (1 to 3) int64 per rank into out[r * k + j] (blocking: the host needs the values)
static int gather_values(kw_comm *c, const int64_t *mine, int k, int64_t *out, hipStream_t st)
{
    if (k < 1 || k > 3) { c->err = "gather_values: 1 to 3 values"; return KW_EINVAL; }
    int64_t *own = c->d_counts + 3 * c->nranks;
    CCHK(c, hipMemcpyAsync(own, mine, sizeof(int64_t) * k, hipMemcpyHostToDevice, st));
    NCHK(c, g_rccl.AllGather(own, c->d_counts, (size_t)k, nccl_int64, c->comm, st));
    CCHK(c, hipMemcpyAsync(out, c->d_counts, sizeof(int64_t) * k * c->nranks, hipMemcpyDeviceToHost, st));
    CCHK(c, hipStreamSynchronize(st));
    return KW_OK;
}

extern "C" int kw_allgather_counts(kw_comm *c, int64_t count, int64_t *counts, void *stream)
{
    if (!c || !counts) return KW_EINVAL;
    CCHK(c, hipSetDevice(c->device));
    return gather_values(c, &count, 1, counts, (hipStream_t)stream);
}

extern "C" int kw_exchange_plan(int32_t nranks, int32_t rank, int32_t root, const int64_t *counts, int64_t *recv_off,
                                int32_t *ops, int64_t *n_total, int64_t *n_recv)
{
    if (nranks < 1 || rank < 0 || rank >= nranks || root >= nranks || !counts || !recv_off || !ops || !n_total ||
        !n_recv)
        return KW_EINVAL;
    recv_off[0] = 0;
    for (int r = 0; r < nranks; ++r) {
        if (counts[r] < 0) return KW_EINVAL;
        recv_off[r + 1] = recv_off[r] + counts[r];
    }
    *n_total = recv_off[nranks];
    const bool receive = root < 0 || root == rank;
    *n_recv = receive ? recv_off[nranks] : 0;
    // point-to-point over the xGMI mesh: every (sender, receiver) pair moves exactly the sender's records;
    // nothing moves to a rank that does not receive, nor from a rank without records
    for (int p = 0; p < nranks; ++p) {
        ops[p] = 0;
        if (p == rank) continue;
        const bool p_receives = root < 0 || root == p;
        if (p_receives && counts[rank] > 0) ops[p] |= KW_PLAN_SEND;
        if (receive && counts[p] > 0) ops[p] |= KW_PLAN_RECV;
    }
    return KW_OK;
}

extern "C" int kw_exchange_caps_ok(int32_t nranks, int32_t root, const int64_t *counts, const int64_t *caps,
                                   int32_t *bad_rank)
{
    if (nranks < 1 || root >= nranks || !counts || !caps) return KW_EINVAL;
    int64_t total = 0;
    for (int r = 0; r < nranks; ++r) {
        if (counts[r] < 0) return KW_EINVAL;
        total += counts[r];
    }
    for (int r = 0; r < nranks; ++r) {
        const bool receives = root < 0 || root == r;
        if (receives && caps[r] < total) {
            if (bad_rank) *bad_rank = r;
            return KW_EOVERFLOW;
        }
    }
    if (bad_rank) *bad_rank = -1;
    return KW_OK;
}

// rebase this rank's n records (into its slot of dst when it receives, else into the staging buffer) and post
// the plan's sends and receives (dst = the receiver's output)
static int post_exchange(kw_comm *c, const kw_hit *d_local, int64_t n, int64_t doc_base, bool receive,
                         const int64_t *pre, const int64_t *cnt, const int32_t *ops, kw_hit *dst, hipStream_t st)
{
    kw_hit *mine = nullptr;
    if (n > 0) {
        if (receive) {
            mine = dst + pre[c->rank];
        } else {
            if ((size_t)n > c->stage_cap) {
                if (c->d_stage) (void)hipFree(c->d_stage);
                c->d_stage = nullptr;
                c->stage_cap = (size_t)n + (size_t)n / 4 + 1024;
                CCHK(c, hipMalloc(&c->d_stage, c->stage_cap * sizeof(kw_hit)));
            }
            mine = c->d_stage;
        }
        const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
        hipLaunchKernelGGL(kw_rebase_kernel, dim3((unsigned)blocks), dim3(256), 0, st, d_local, mine, n, (uint32_t)doc_base);
        CCHK(c, hipGetLastError());
    }
    if (c->nranks == 1) return KW_OK;
    // point-to-point over the xGMI mesh: every (sender, receiver) pair moves exactly its records
    NCHK(c, g_rccl.GroupStart());
    for (int p = 0; p < c->nranks; ++p) {
        if (ops[p] & KW_PLAN_SEND) NCHK(c, g_rccl.Send(mine, (size_t)n * 4, nccl_uint32, p, c->comm, st));
        if (ops[p] & KW_PLAN_RECV) NCHK(c, g_rccl.Recv(dst + pre[p], (size_t)cnt[p] * 4, nccl_uint32, p, c->comm, st));
    }
    NCHK(c, g_rccl.GroupEnd());
    return KW_OK;
}

extern "C" int kw_allgather_hits(kw_comm *c, const kw_hit *d_local, int64_t n, int64_t doc_base, int32_t root,
                                 kw_hit *d_out, int64_t cap, int64_t *n_total, int64_t *counts, void *stream)
{
    if (!c || !n_total || n < 0 || (n > 0 && !d_local)) return KW_EINVAL;
    if (root >= c->nranks || doc_base < 0) { c->err = "kw_allgather_hits: bad root or doc_base"; return KW_EINVAL; }
    hipStream_t st = (hipStream_t)stream;
    CCHK(c, hipSetDevice(c->device));
    const bool receive = root < 0 || root == c->rank;
    // one exchange of (count, receiver capacity, error) triples: every rank sees every receiver's room and every
    // rank's local verdict, so a short destination or a rank whose global document ids overflow 32 bits fails on
    // EVERY rank here, before any record moves (no peer is left waiting in a send)
    const int64_t bad_ids = doc_base + n > 0xFFFFFFFFll ? 1 : 0;
    const int64_t mine[3] = {n, receive ? (d_out ? cap : 0) : INT64_MAX, bad_ids};
    std::vector<int64_t> trip((size_t)3 * c->nranks);
    int rc = gather_values(c, mine, 3, trip.data(), st);
    if (rc) return rc;
    std::vector<int64_t> cnt(c->nranks), caps(c->nranks);
    for (int r = 0; r < c->nranks; ++r) {
        cnt[r] = trip[3 * r];
        caps[r] = trip[3 * r + 1];
    }
    for (int r = 0; r < c->nranks; ++r) {
        if (trip[3 * r + 2]) {
            char buf[160];
            snprintf(buf, sizeof(buf), "kw_allgather_hits: rank %d's global document ids go beyond 2^32", r);
            c->err = buf;
            return KW_EINVAL;
        }
    }
    std::vector<int64_t> pre(c->nranks + 1, 0);
    std::vector<int32_t> ops(c->nranks, 0);
    int64_t n_recv = 0;
    if (kw_exchange_plan(c->nranks, c->rank, root, cnt.data(), pre.data(), ops.data(), n_total, &n_recv) != KW_OK) {
        c->err = "kw_allgather_hits: bad exchange plan";
        return KW_EINVAL;
    }
    if (counts) memcpy(counts, cnt.data(), sizeof(int64_t) * c->nranks);
    int32_t bad = -1;
    if (kw_exchange_caps_ok(c->nranks, root, cnt.data(), caps.data(), &bad) != KW_OK) {
        char buf[160];
        snprintf(buf, sizeof(buf), "kw_allgather_hits: rank %d's destination holds %lld records, the exchange has %lld",
                 bad, (long long)caps[bad], (long long)*n_total);
        c->err = buf;
        return KW_EOVERFLOW;
    }
    return post_exchange(c, d_local, n, doc_base, receive, pre.data(), cnt.data(), ops.data(), d_out, st);
}

extern "C" int kw_allgather_hits_planned(kw_comm *c, const kw_hit *d_local, int64_t n, int64_t doc_base, int32_t root,
                                         const int64_t *counts, kw_hit *d_out, int64_t cap, int64_t *n_total,
                                         void *stream)
{
    if (!c || !n_total || !counts || n < 0 || (n > 0 && !d_local)) return KW_EINVAL;
    if (root >= c->nranks || doc_base < 0) { c->err = "kw_allgather_hits_planned: bad root or doc_base"; return KW_EINVAL; }
    hipStream_t st = (hipStream_t)stream;
    CCHK(c, hipSetDevice(c->device));
    std::vector<int64_t> pre(c->nranks + 1, 0);
    std::vector<int32_t> ops(c->nranks, 0);
    int64_t n_recv = 0;
    // (the same counts on every rank: a negative count -- kw_allgather_counts' error flag -- fails every rank here,
    // before anything is posted)
    if (kw_exchange_plan(c->nranks, c->rank, root, counts, pre.data(), ops.data(), n_total, &n_recv) != KW_OK) {
        c->err = "kw_allgather_hits_planned: bad counts (a rank flagged an error with a negative count)";
        return KW_EINVAL;
    }
    const char *local_err = nullptr;
    if (counts[c->rank] != n) local_err = "kw_allgather_hits_planned: counts[rank] is not this rank's n";
    else if (doc_base + n > 0xFFFFFFFFll) local_err = "kw_allgather_hits_planned: global document ids beyond 2^32";
    if (local_err) {
        // the peers already post their halves from `counts`: post this rank's matching sends and receives (zero
        // records of the agreed size from / into the library's buffer) so no one waits, then fail this rank
        const int64_t need = std::max<int64_t>(counts[c->rank], n_recv);
        if ((size_t)need > c->spill_cap) {
            if (c->d_spill) (void)hipFree(c->d_spill);
            c->d_spill = nullptr;
            c->spill_cap = (size_t)need;
            CCHK(c, hipMalloc(&c->d_spill, c->spill_cap * sizeof(kw_hit)));
        }
        if (need > 0) CCHK(c, hipMemsetAsync(c->d_spill, 0, (size_t)need * sizeof(kw_hit), st));
        if (c->nranks > 1) {
            NCHK(c, g_rccl.GroupStart());
            for (int p = 0; p < c->nranks; ++p) {
                if (ops[p] & KW_PLAN_SEND)
                    NCHK(c, g_rccl.Send(c->d_spill, (size_t)counts[c->rank] * 4, nccl_uint32, p, c->comm, st));
                if (ops[p] & KW_PLAN_RECV)
                    NCHK(c, g_rccl.Recv(c->d_spill, (size_t)counts[p] * 4, nccl_uint32, p, c->comm, st));
            }
            NCHK(c, g_rccl.GroupEnd());
        }
        c->err = local_err;
        return KW_EINVAL;
    }
    const bool receive = root < 0 || root == c->rank;
    kw_hit *dst = d_out;
    bool short_dst = false;
    if (receive && (n_recv > cap || (n_recv > 0 && !d_out))) {
        // every peer already posts its sends from the same counts: receive into the library's buffer so no one
        // waits, then report the short destination (the records are dropped)
        if ((size_t)n_recv > c->spill_cap) {
            if (c->d_spill) (void)hipFree(c->d_spill);
            c->d_spill = nullptr;
            c->spill_cap = (size_t)n_recv;
            CCHK(c, hipMalloc(&c->d_spill, c->spill_cap * sizeof(kw_hit)));
        }
        dst = c->d_spill;
        short_dst = true;
    }
    int rc = post_exchange(c, d_local, n, doc_base, receive, pre.data(), counts, ops.data(), dst, st);
    if (rc) return rc;
    if (short_dst) {
        c->err = "kw_allgather_hits_planned: destination too small (records received into a library buffer and dropped)";
        return KW_EOVERFLOW;
    }
    return KW_OK;
}

extern "C" const char *kw_comm_last_error(kw_comm *c)
{
    return c ? c->err.c_str() : g_comm_err.c_str();
}

extern "C" int kw_comm_destroy(kw_comm *c)
{
    if (!c) return KW_OK;
    (void)hipSetDevice(c->device);
    if (c->comm) (void)g_rccl.CommDestroy(c->comm);
    if (c->d_counts) (void)hipFree(c->d_counts);
    if (c->d_stage) (void)hipFree(c->d_stage);
    if (c->d_spill) (void)hipFree(c->d_spill);
    delete c;
    return KW_OK;
}
