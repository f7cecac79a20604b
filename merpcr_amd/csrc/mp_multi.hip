// Multi-GPU search: one genome's (sequence, k) space split into owned ranges, one range
// per device, and the per-device sorted hit lists gathered into one list over xGMI.
//
// every window position is independent and owned ranges are contiguous in
// (sequence, k), so the rank-ordered concatenation of the per-device sorted lists is the
// reference's output order (engine.py:434, T=1 semantics); boundary tests inside each
// device use the true sequence lengths (the whole layout is known to every device), so
// the union is exactly the single-device result.  The reference's own parallelism is
// the -T ProcessPool fan-out over chunks of one record (engine.py:386-422); this replaces
// it.
//
// Two forms:
//   * mp_multi_*: one process drives several devices: a host thread per device for the
//     pack, the searches enqueued and completed from the calling thread (they run
//     concurrently), then the copy engines move every device's list into devices[0]
//     (hipMemcpyPeerAsync on devices[0]'s stream; a repeated device -- tests on one GPU --
//     takes the very same copies).  A grouped ncclSend/ncclRecv gatherv stays behind
//     mp_multi_set_gather(MP_GATHER_RCCL), distinct devices only.
//   * mp_comm_*: one process per GPU (torchrun / MPI style): the caller shares the RCCL
//     unique id out of band; every rank's last search result is gathered to rank 0.
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "mp_internal.h"

namespace mp {

#define MP_NCCL_CHECK(expr)                                                              \
    do {                                                                                 \
        ncclResult_t _r = (expr);                                                        \
        if (_r != ncclSuccess)                                                           \
            return ::mp::fail(MP_E_HIP, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
    } while (0)

// seq += shift[segment] for the gathered hits of each rank (contig shards of a larger
// record set: each rank numbers its sequences from 0)
__global__ void shift_seq_kernel(mp_hit* __restrict__ h, uint64_t n, uint32_t shift) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) h[i].seq += shift;
}

struct Multi {
    std::vector<int> dev;
    std::vector<Table*> tab;
    std::vector<Genome*> gen;
    std::vector<Search*> srch;
    std::vector<hipStream_t> st;
    std::vector<ncclComm_t> comm;   // MP_GATHER_RCCL only (made at its first run)
    int gather = MP_GATHER_COPY;
    bool distinct = false;          // no device listed twice
    std::vector<mp_range> rng;      // owned range per device
    std::vector<std::vector<std::pair<uint64_t, uint64_t>>> need;  // per device, per sequence: bases packed
    std::vector<uint64_t> counts;
    std::vector<uint64_t> len;
    mp_hit* all = nullptr;          // gathered hits on dev[0]
    uint64_t all_cap = 0, n_all = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;  // gather timing on dev[0], made once
    hipEvent_t es = nullptr;                // the call's start on dev[0] (span: es -> e1)
    float span_ms = 0.f;
    std::vector<hipEvent_t> sent;           // per device: its gather send is queued (RCCL form)
    float gather_ms = 0.f;
};

static void free_multi(Multi* m) {
    if (!m) return;
    for (auto c : m->comm) ncclCommDestroy(c);
    for (size_t i = 0; i < m->dev.size(); ++i) {
        hipSetDevice(m->dev[i]);
        if (m->srch[i]) mp_search_destroy(m->srch[i]);
        if (i < m->sent.size() && m->sent[i]) hipEventDestroy(m->sent[i]);
        if (m->gen[i]) mp_genome_destroy(m->gen[i]);
        if (m->st[i]) hipStreamDestroy(m->st[i]);
    }
    if (!m->dev.empty()) {
        hipSetDevice(m->dev[0]);
        if (m->all) hipFree(m->all);
        if (m->e0) hipEventDestroy(m->e0);
        if (m->e1) hipEventDestroy(m->e1);
        if (m->es) hipEventDestroy(m->es);
    }
    delete m;
}

// Owned (sequence, k) ranges of equal base count, in order; the last ends at the genome's end.
static void split_ranges(const std::vector<uint64_t>& len, uint32_t parts, std::vector<mp_range>& out) {
    uint64_t total = 0;
    for (auto l : len) total += l;
    const uint32_t n_seq = (uint32_t)len.size();
    out.assign(parts, mp_range{0, 0, 0, 0});
    uint32_t q = 0;
    uint64_t before = 0;  // bases of sequences < q
    mp_range cur{0, 0, 0, 0};
    for (uint32_t p = 0; p < parts; ++p) {
        out[p].seq_begin = cur.seq_begin;
        out[p].k_begin = cur.k_begin;
        if (p + 1 == parts) {
            out[p].seq_end = n_seq;
            out[p].k_end = 0;
            break;
        }
        const uint64_t cut = total * (p + 1) / parts;  // global base index of the cut
        while (q < n_seq && before + len[q] <= cut) {
            before += len[q];
            ++q;
        }
        out[p].seq_end = q;
        out[p].k_end = q < n_seq ? cut - before : 0;
        cur.seq_begin = q;
        cur.k_begin = out[p].k_end;
    }
}

// Run fn(d) for every device in a host thread of its own; the first failure is re-raised
// on the calling thread (error messages are thread-local).
template <class F>
static int per_device(uint32_t nd, F&& fn) {
    std::vector<int> rc(nd, MP_OK);
    std::vector<std::string> msg(nd);
    std::vector<std::thread> th;
    for (uint32_t d = 0; d < nd; ++d)
        th.emplace_back([&, d] {
            rc[d] = fn(d);
            if (rc[d]) msg[d] = mp_last_error();
        });
    for (auto& x : th) x.join();
    for (uint32_t d = 0; d < nd; ++d)
        if (rc[d]) return fail(rc[d], msg[d]);
    return MP_OK;
}

static int multi_layout(Multi* m, uint32_t n_seq, const uint64_t* seq_len) {
    const uint32_t nd = (uint32_t)m->dev.size();
    m->len.assign(seq_len, seq_len + n_seq);
    split_ranges(m->len, nd, m->rng);
    m->need.assign(nd, std::vector<std::pair<uint64_t, uint64_t>>(n_seq, {0, 0}));
    for (uint32_t d = 0; d < nd; ++d) {
        const mp_range& r = m->rng[d];
        const uint64_t halo = m->tab[d]->max_reach + 64;  // bases past an owned k any compare reads
        for (uint32_t q = r.seq_begin; q < n_seq && q <= r.seq_end; ++q) {
            const uint64_t lo = q == r.seq_begin ? r.k_begin : 0;
            const uint64_t hi = q == r.seq_end ? r.k_end : m->len[q];
            if (hi <= lo) continue;
            const uint64_t a = lo & ~63ull;
            uint64_t b = std::min<uint64_t>(m->len[q], hi + halo + m->tab[d]->max_hash_off);
            if (b < m->len[q]) b = std::min<uint64_t>(m->len[q], round_up(b, 64));
            m->need[d][q] = {a, b};
        }
    }
    // one thread per device: (re)lay every device's genome out on its own buffers
    return per_device(nd, [&](uint32_t d) -> int {
        if (hipSetDevice(m->dev[d]) != hipSuccess) return fail(MP_E_HIP, "hipSetDevice failed");
        if (m->gen[d]) return mp_genome_reset(m->gen[d], n_seq, seq_len);
        void* g = nullptr;
        int rc = mp_genome_create(m->dev[d], n_seq, seq_len, &g);
        m->gen[d] = (Genome*)g;
        if (rc) return rc;
        void* s = nullptr;
        rc = mp_search_create(m->tab[d], m->gen[d], &s);
        m->srch[d] = (Search*)s;
        return rc;
    });
}

}  // namespace mp

using namespace mp;

MP_EXPORT int mp_multi_create(uint32_t n_dev, const int32_t* devices, void* const* tables, void** out) {
    if (!out || !n_dev || !devices || !tables) return fail(MP_E_ARG, "mp_multi_create: null pointer or no device");
    *out = nullptr;
    Multi* m = new Multi();
    m->dev.assign(devices, devices + n_dev);
    m->tab.resize(n_dev);
    m->gen.assign(n_dev, nullptr);
    m->srch.assign(n_dev, nullptr);
    m->st.assign(n_dev, nullptr);
    m->counts.assign(n_dev, 0);
    m->sent.assign(n_dev, nullptr);
    int rc = MP_OK;
    for (uint32_t d = 0; d < n_dev && !rc; ++d) {
        m->tab[d] = (Table*)tables[d];
        if (!m->tab[d]) rc = fail(MP_E_ARG, "mp_multi_create: null table");
        else if (m->tab[d]->device != m->dev[d]) rc = fail(MP_E_ARG, "mp_multi_create: table i must live on devices[i]");
        else if (hipSetDevice(m->dev[d]) != hipSuccess || hipStreamCreateWithFlags(&m->st[d], hipStreamNonBlocking) != hipSuccess ||
                 hipEventCreateWithFlags(&m->sent[d], hipEventDisableTiming) != hipSuccess)
            rc = fail(MP_E_HIP, "mp_multi_create: stream creation failed");
    }
    if (!rc && (hipSetDevice(m->dev[0]) != hipSuccess || hipEventCreate(&m->e0) != hipSuccess ||
                hipEventCreate(&m->e1) != hipSuccess || hipEventCreate(&m->es) != hipSuccess))
        rc = fail(MP_E_HIP, "mp_multi_create: event creation failed");
    if (!rc) {
        std::vector<int> sorted(m->dev);
        std::sort(sorted.begin(), sorted.end());
        m->distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
        // the gather's copies run on devices[0]'s stream and read the other devices' lists:
        // direct xGMI reads need peer access from devices[0] (without it HIP stages the copy)
        (void)hipSetDevice(m->dev[0]);
        for (uint32_t d = 1; d < n_dev; ++d) {
            int can = 0;
            if (m->dev[d] != m->dev[0] && hipDeviceCanAccessPeer(&can, m->dev[0], m->dev[d]) == hipSuccess && can) {
                const hipError_t e = hipDeviceEnablePeerAccess(m->dev[d], 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                    rc = fail(MP_E_HIP, std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorString(e));
                (void)hipGetLastError();  // an "already enabled" error is not sticky for later calls
            }
        }
    }
    if (rc) {
        free_multi(m);
        return rc;
    }
    *out = m;
    return MP_OK;
}

MP_EXPORT int mp_multi_set_gather(void* multi, int32_t mode) {
    Multi* m = (Multi*)multi;
    if (!m) return fail(MP_E_ARG, "mp_multi_set_gather: null multi");
    if (mode != MP_GATHER_COPY && mode != MP_GATHER_RCCL) return fail(MP_E_ARG, "mp_multi_set_gather: unknown mode");
    if (mode == MP_GATHER_RCCL && !m->distinct)
        return fail(MP_E_ARG, "mp_multi_set_gather: RCCL admits one rank per device (a device is listed twice)");
    if (mode == MP_GATHER_RCCL && m->comm.empty()) {
        m->comm.resize(m->dev.size());
        const ncclResult_t r = ncclCommInitAll(m->comm.data(), (int)m->dev.size(), m->dev.data());
        if (r != ncclSuccess) {
            m->comm.clear();
            return fail(MP_E_HIP, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
        }
    }
    m->gather = mode;
    return MP_OK;
}

MP_EXPORT int mp_multi_genome(void* multi, uint32_t n_seq, const uint64_t* seq_len) {
    Multi* m = (Multi*)multi;
    if (!m || (n_seq && !seq_len)) return fail(MP_E_ARG, "mp_multi_genome: null pointer");
    return multi_layout(m, n_seq, seq_len);
}

MP_EXPORT int mp_multi_put(void* multi, uint32_t seq, const uint8_t* host_bytes, uint64_t nbytes) {
    Multi* m = (Multi*)multi;
    if (!m || (nbytes && !host_bytes)) return fail(MP_E_ARG, "mp_multi_put: null pointer");
    if (seq >= m->len.size()) return fail(MP_E_ARG, "mp_multi_put: sequence index out of range");
    if (nbytes != m->len[seq]) return fail(MP_E_ARG, "mp_multi_put: pass the whole sequence");
    return per_device((uint32_t)m->dev.size(), [&](uint32_t d) -> int {
        const auto [a, b] = m->need[d][seq];  // each device packs the part its owned range reads
        return b > a ? mp_genome_put(m->gen[d], seq, a, host_bytes + a, b - a, m->st[d]) : MP_OK;
    });
}

MP_EXPORT int mp_multi_seal(void* multi) {
    Multi* m = (Multi*)multi;
    if (!m) return fail(MP_E_ARG, "mp_multi_seal: null multi");
    return per_device((uint32_t)m->dev.size(), [&](uint32_t d) { return mp_genome_seal(m->gen[d], m->st[d]); });
}

// Every device's run is enqueued from the calling thread (mp_search_enqueue returns as soon as
// its kernels are queued), then completed device by device (each polls its own run's event),
// so the devices search concurrently with no host thread started per call.  The gather waits
// on the devices, not the host: device 0's stream takes every sender's event before the
// gather-end event the host polls.  (Round 3 started a std::thread per device per call and
// synchronised every device's stream.)
MP_EXPORT int mp_multi_run(void* multi, uint64_t* n_hits) {
    Multi* m = (Multi*)multi;
    if (!m) return fail(MP_E_ARG, "mp_multi_run: null multi");
    if (!m->gen[0]) return fail(MP_E_STATE, "mp_multi_run: no genome (call mp_multi_genome)");
    const uint32_t nd = (uint32_t)m->dev.size();
    if (n_hits) *n_hits = 0;
    MP_HIP_CHECK(hipSetDevice(m->dev[0]));
    MP_HIP_CHECK(hipEventRecord(m->es, m->st[0]));
    for (uint32_t d = 0; d < nd; ++d) {
        const int rc = mp_search_enqueue(m->srch[d], &m->rng[d], m->st[d]);
        if (rc) {
            for (uint32_t e = 0; e < d; ++e) mp_search_complete(m->srch[e], nullptr);  // drain what was queued
            return rc;
        }
    }
    int rc = MP_OK;
    std::string msg;
    for (uint32_t d = 0; d < nd; ++d) {  // complete them all, keeping the first failure
        const int r = mp_search_complete(m->srch[d], &m->counts[d]);
        if (r && !rc) {
            rc = r;
            msg = mp_last_error();
        }
    }
    if (rc) return fail(rc, msg);
    uint64_t total = 0;
    for (auto c : m->counts) total += c;
    MP_HIP_CHECK(hipSetDevice(m->dev[0]));
    if (total > m->all_cap) {
        hipFree(m->all);
        m->all = nullptr;
        m->all_cap = 0;
        const uint64_t cap = total + total / 4 + 1024;
        MP_HIP_CHECK(hipMalloc(&m->all, cap * sizeof(mp_hit)));
        m->all_cap = cap;
    }
    MP_HIP_CHECK(hipEventRecord(m->e0, m->st[0]));
    uint64_t off = 0;
    if (m->gather == MP_GATHER_RCCL) {
        // gatherv over RCCL: devices[0] receives every device's sorted list at its offset
        MP_NCCL_CHECK(ncclGroupStart());
        for (uint32_t d = 0; d < nd; ++d) {
            const size_t bytes = m->counts[d] * sizeof(mp_hit);
            if (bytes) {
                MP_NCCL_CHECK(ncclRecv(m->all + off, bytes, ncclUint8, (int)d, m->comm[0], m->st[0]));
                MP_NCCL_CHECK(ncclSend(m->srch[d]->out, bytes, ncclUint8, 0, m->comm[d], m->st[d]));
            }
            off += m->counts[d];
        }
        MP_NCCL_CHECK(ncclGroupEnd());
        // device 0's stream waits (on the device) for every sender; a sender's next run is
        // queued behind its send on its own stream
        for (uint32_t d = 1; d < nd; ++d) {
            MP_HIP_CHECK(hipSetDevice(m->dev[d]));
            MP_HIP_CHECK(hipEventRecord(m->sent[d], m->st[d]));
        }
        MP_HIP_CHECK(hipSetDevice(m->dev[0]));
        for (uint32_t d = 1; d < nd; ++d) MP_HIP_CHECK(hipStreamWaitEvent(m->st[0], m->sent[d], 0));
    } else {
        // the copy engines, one peer copy per device on devices[0]'s stream (xGMI between
        // distinct devices, a local copy for a repeated one): every run was completed above,
        // so each list is final; no kernel on the CUs
        for (uint32_t d = 0; d < nd; ++d) {
            const size_t bytes = m->counts[d] * sizeof(mp_hit);
            if (bytes)
                MP_HIP_CHECK(hipMemcpyPeerAsync(m->all + off, m->dev[0], m->srch[d]->out, m->dev[d], bytes, m->st[0]));
            off += m->counts[d];
        }
    }
    MP_HIP_CHECK(hipEventRecord(m->e1, m->st[0]));
    MP_HIP_CHECK(poll_event(m->e1));
    MP_HIP_CHECK(hipEventElapsedTime(&m->gather_ms, m->e0, m->e1));
    MP_HIP_CHECK(hipEventElapsedTime(&m->span_ms, m->es, m->e1));
    m->n_all = total;
    if (n_hits) *n_hits = total;
    return MP_OK;
}

MP_EXPORT int mp_multi_fetch(void* multi, mp_hit* out, uint64_t cap) {
    Multi* m = (Multi*)multi;
    if (!m || (m->n_all && !out)) return fail(MP_E_ARG, "mp_multi_fetch: null pointer");
    if (cap < m->n_all) return fail(MP_E_CAP, "mp_multi_fetch: output buffer too small");
    if (!m->n_all) return MP_OK;
    MP_HIP_CHECK(hipSetDevice(m->dev[0]));
    MP_HIP_CHECK(hipMemcpyAsync(out, m->all, m->n_all * sizeof(mp_hit), hipMemcpyDeviceToHost, m->st[0]));
    MP_HIP_CHECK(hipStreamSynchronize(m->st[0]));
    return MP_OK;
}

MP_EXPORT int mp_multi_device_search(void* multi, uint32_t i, void** search, mp_range* owned, float* gather_ms) {
    Multi* m = (Multi*)multi;
    if (!m || i >= m->dev.size()) return fail(MP_E_ARG, "mp_multi_device_search: bad index");
    if (search) *search = m->srch[i];
    if (owned) *owned = i < m->rng.size() ? m->rng[i] : mp_range{0, 0, 0, 0};
    if (gather_ms) *gather_ms = m->gather_ms;
    return MP_OK;
}

MP_EXPORT int mp_multi_timing(void* multi, float* span_ms, float* gather_ms) {
    Multi* m = (Multi*)multi;
    if (!m) return fail(MP_E_ARG, "mp_multi_timing: null multi");
    if (span_ms) *span_ms = m->span_ms;
    if (gather_ms) *gather_ms = m->gather_ms;
    return MP_OK;
}

MP_EXPORT void mp_multi_destroy(void* multi) { free_multi((Multi*)multi); }

// ---------------------------------------------------------------- process per GPU
namespace mp {
struct Comm {
    ncclComm_t c = nullptr;
    int rank = 0, nranks = 1, device = 0;
    uint64_t* d_meta = nullptr;  // nranks x {count, seq shift, capacity}
    uint64_t* h_meta = nullptr;  // pinned: this rank's 3 words, then the gathered nranks x 3
    hipEvent_t ev = nullptr;     // the gathered counts' arrival (polled)
    double timeout_s = 600.0;    // MP_COMM_TIMEOUT_S: bound on waiting for the other ranks
};
}  // namespace mp

static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id is 128 bytes");

MP_EXPORT int mp_comm_unique_id(uint8_t* id) {
    if (!id) return fail(MP_E_ARG, "mp_comm_unique_id: null pointer");
    ncclUniqueId u;
    MP_NCCL_CHECK(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof(u));
    return MP_OK;
}

MP_EXPORT int mp_comm_create(const uint8_t* id, int32_t nranks, int32_t rank, int32_t device, void** out) {
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) return fail(MP_E_ARG, "mp_comm_create: bad argument");
    *out = nullptr;
    MP_HIP_CHECK(hipSetDevice(device));
    Comm* c = new Comm();
    if (const char* t = std::getenv("MP_COMM_TIMEOUT_S")) c->timeout_s = std::atof(t);
    c->rank = rank;
    c->nranks = nranks;
    c->device = device;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclResult_t r = ncclCommInitRank(&c->c, nranks, u, rank);
    if (r != ncclSuccess) {
        delete c;
        return fail(MP_E_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    if (hipMalloc(&c->d_meta, (size_t)nranks * 3 * sizeof(uint64_t)) != hipSuccess ||
        hipHostMalloc((void**)&c->h_meta, (size_t)(nranks + 1) * 3 * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev, hipEventDisableTiming) != hipSuccess) {
        hipFree(c->d_meta);
        if (c->h_meta) hipHostFree(c->h_meta);
        ncclCommDestroy(c->c);
        delete c;
        return fail(MP_E_NOMEM, "mp_comm_create: allocation failed");
    }
    *out = c;
    return MP_OK;
}

// Gatherv of every rank's last-run hits (mp_search_run on `search`) to rank 0, in rank
// order, into dev_out (rank 0's device, cap entries).  Each rank names the shift of its
// sequence indices (its first record in the caller's global numbering).  Collective:
// every rank calls it; *n_total = all ranks' hits on every rank; MP_E_CAP on every rank
// when rank 0's cap is too small (nothing is sent then).
MP_EXPORT int mp_comm_gather_hits(void* comm, void* search, uint32_t seq_shift, mp_hit* dev_out, uint64_t cap,
                                  uint64_t* n_total, void* stream) {
    Comm* c = (Comm*)comm;
    Search* s = (Search*)search;
    if (!c || !s || !n_total || (c->rank == 0 && cap && !dev_out)) return fail(MP_E_ARG, "mp_comm_gather_hits: null pointer");
    hipStream_t st = (hipStream_t)stream;
    MP_HIP_CHECK(hipSetDevice(c->device));
    // pinned staging and a polled event: the counts exchange is on every step's critical path
    uint64_t* mine = c->h_meta;
    const uint64_t* meta = c->h_meta + 3;
    // a rank whose run is still enqueued (hit list being written) sends the marker ~0: every
    // rank then leaves with MP_E_STATE after the counts exchange, so no rank waits on it
    mine[0] = s->pending ? ~0ull : s->n_hits;
    mine[1] = seq_shift;
    mine[2] = cap;
    MP_HIP_CHECK(hipMemcpyAsync(c->d_meta + (size_t)c->rank * 3, mine, 3 * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    MP_NCCL_CHECK(ncclAllGather(c->d_meta + (size_t)c->rank * 3, c->d_meta, 3, ncclUint64, c->c, st));
    MP_HIP_CHECK(hipMemcpyAsync(c->h_meta + 3, c->d_meta, (size_t)c->nranks * 3 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    MP_HIP_CHECK(hipEventRecord(c->ev, st));
    {
        const hipError_t e = poll_event(c->ev, c->timeout_s);
        if (e == hipErrorNotReady)
            return fail(MP_E_HIP, "mp_comm_gather_hits: the counts exchange did not complete within the "
                                  "timeout (a rank missing from the collective?)");
        MP_HIP_CHECK(e);
    }
    uint64_t total = 0;
    for (int r = 0; r < c->nranks; ++r)
        if (meta[(size_t)r * 3] == ~0ull)
            return fail(MP_E_STATE, "mp_comm_gather_hits: a rank's search run is enqueued (mp_search_complete first)");
    for (int r = 0; r < c->nranks; ++r) total += meta[(size_t)r * 3];
    *n_total = total;
    if (total > meta[2]) return fail(MP_E_CAP, "mp_comm_gather_hits: rank 0 buffer too small");
    MP_NCCL_CHECK(ncclGroupStart());
    uint64_t off = 0;
    for (int r = 0; r < c->nranks; ++r) {
        const size_t bytes = meta[(size_t)r * 3] * sizeof(mp_hit);
        if (bytes) {
            if (c->rank == 0) MP_NCCL_CHECK(ncclRecv(dev_out + off, bytes, ncclUint8, r, c->c, st));
            if (c->rank == r) MP_NCCL_CHECK(ncclSend(s->out, bytes, ncclUint8, 0, c->c, st));
        }
        off += meta[(size_t)r * 3];
    }
    MP_NCCL_CHECK(ncclGroupEnd());
    if (c->rank == 0) {
        off = 0;
        for (int r = 0; r < c->nranks; ++r) {
            const uint64_t n = meta[(size_t)r * 3];
            const uint32_t sh = (uint32_t)meta[(size_t)r * 3 + 1];
            if (n && sh) {
                hipLaunchKernelGGL(shift_seq_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, dev_out + off, n, sh);
                MP_HIP_CHECK(hipGetLastError());
            }
            off += n;
        }
    }
    return MP_OK;
}

MP_EXPORT void mp_comm_destroy(void* comm) {
    Comm* c = (Comm*)comm;
    if (!c) return;
    hipSetDevice(c->device);
    hipFree(c->d_meta);
    if (c->h_meta) hipHostFree(c->h_meta);
    if (c->ev) hipEventDestroy(c->ev);
    if (c->c) ncclCommDestroy(c->c);
    delete c;
}

// ---- hit gather by the copy engines (one node; include/merpcr_hip.h)
static_assert(sizeof(hipIpcMemHandle_t) == MP_IPC_HANDLE_BYTES, "IPC handle size");

MP_EXPORT int mp_ipc_handle(void* dev_ptr, uint8_t* handle64, uint64_t* offset) {
    if (!dev_ptr || !handle64 || !offset) return fail(MP_E_ARG, "mp_ipc_handle: null pointer");
    // the handle names the whole allocation (a caching allocator's block may hold several
    // buffers): the importer maps its base and adds dev_ptr's offset in it
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    MP_HIP_CHECK(hipMemGetAddressRange(&base, &size, dev_ptr));
    *offset = (uint64_t)((const char*)dev_ptr - (const char*)base);
    hipIpcMemHandle_t h;
    MP_HIP_CHECK(hipIpcGetMemHandle(&h, dev_ptr));
    std::memcpy(handle64, &h, sizeof(h));
    return MP_OK;
}

MP_EXPORT int mp_ipc_open(const uint8_t* handle64, int32_t device, void** dev_ptr_out) {  // the allocation's base
    if (!handle64 || !dev_ptr_out) return fail(MP_E_ARG, "mp_ipc_open: null pointer");
    *dev_ptr_out = nullptr;
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle64, sizeof(h));
    MP_HIP_CHECK(hipSetDevice(device));
    MP_HIP_CHECK(hipIpcOpenMemHandle(dev_ptr_out, h, hipIpcMemLazyEnablePeerAccess));
    return MP_OK;
}

MP_EXPORT int mp_ipc_close(void* dev_ptr) {
    if (!dev_ptr) return fail(MP_E_ARG, "mp_ipc_close: null pointer");
    MP_HIP_CHECK(hipIpcCloseMemHandle(dev_ptr));
    return MP_OK;
}

// The count travels from a pinned ring slot (kPutRing per handle); a slot is reused only after
// the copy that read it has run (its event), and the handle's next run waits on the device for
// the hit copy (put_done, taken by mp_search_enqueue on whatever stream that run uses).
MP_EXPORT int mp_search_put_hits(void* search, mp_hit* dst, uint64_t cap, uint64_t* count_dst, uint64_t* n_hits,
                                 void* stream) {
    Search* s = (Search*)search;
    if (n_hits) *n_hits = s ? s->n_hits : 0;
    if (!s || !count_dst || (s->n_hits && !dst)) return fail(MP_E_ARG, "mp_search_put_hits: null pointer");
    if (s->pending) return fail(MP_E_STATE, "mp_search_put_hits: a run is enqueued (mp_search_complete first)");
    if (s->n_hits > cap) return fail(MP_E_CAP, "mp_search_put_hits: region too small (*n_hits = the need)");
    hipStream_t st = (hipStream_t)stream;
    MP_HIP_CHECK(hipSetDevice(s->genome->device));
    if (!s->h_put) {
        MP_HIP_CHECK(hipHostMalloc((void**)&s->h_put, kPutRing * sizeof(unsigned long long), hipHostMallocDefault));
        s->put_ev = new hipEvent_t[kPutRing]();
        for (uint32_t i = 0; i < kPutRing; ++i)
            MP_HIP_CHECK(hipEventCreateWithFlags(&s->put_ev[i], hipEventDisableTiming));
        MP_HIP_CHECK(hipEventCreateWithFlags(&s->put_done, hipEventDisableTiming));
    }
    const uint64_t n = s->n_hits;
    if (n) MP_HIP_CHECK(hipMemcpyAsync(dst, s->out, n * sizeof(mp_hit), hipMemcpyDeviceToDeviceNoCU, st));
    MP_HIP_CHECK(hipEventRecord(s->put_done, st));
    s->put_wait = true;
    const uint32_t k = s->put_seq++ % kPutRing;
    if (s->put_seq > kPutRing) MP_HIP_CHECK(hipEventSynchronize(s->put_ev[k]));  // kPutRing puts ago: long done
    unsigned long long* c = s->h_put + k;
    *c = n;
    MP_HIP_CHECK(hipMemcpyAsync(count_dst, c, sizeof(uint64_t), hipMemcpyHostToDevice, st));
    MP_HIP_CHECK(hipEventRecord(s->put_ev[k], st));
    return MP_OK;
}
