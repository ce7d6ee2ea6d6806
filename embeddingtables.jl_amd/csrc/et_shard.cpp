// et_shard.cpp — the sharded PreallocationStrategy step (BASELINE config 5) behind the
// C ABI: the shard plan, an RCCL communicator, and the pipelined lookup -> all-gather ->
// assembly loop, host-side C++ over the library's own kernels (et_maplookup_prealloc,
// et_concat_slabs, et_split_slabs) and RCCL over xGMI.
//
// No counterpart exists in the single-process reference: this replaces the concat that
// maplookup!(::PreallocationStrategy, dst, tables, I) performs by writing every table's
// lookup into its row block of one destination (src/lookup.jl:316-371, the views at
// :334-340) when the tables live on different GPUs.  The Julia host reaches it through
// the same ccall layer as the single-GPU entry points.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <map>
#include <mutex>
#include <new>
#include <set>
#include <vector>

#include "et_common.h"

namespace et {

#define ET_NCCL_CHECK(call)                                                             \
    do {                                                                                \
        ncclResult_t r_ = (call);                                                       \
        if (r_ != ncclSuccess)                                                          \
            return ::et::fail(ET_ERR_HIP, "%s failed: %s", #call, ncclGetErrorString(r_)); \
    } while (0)

// ---------------------------------------------------------------------------------------
// Recycled events and side streams.  A caller's stream that waited on one of our events
// (the sharded step's join, a loopback rank's copies) may be a pooled stream the caller
// reuses long after the step or the group is gone (torch hands out 32 pooled streams per
// priority round-robin); destroying the event then was followed, tests later, by a
// segmentation fault inside hipGraphLaunch of a capture on such a stream (full GPU suite,
// round 6).  So the runtime never destroys the events and streams it hands to callers'
// streams: et_sharded_destroy / et_comm_destroy return them to a per-device free list that
// later steps and groups take from (bounded by the peak number alive at once).
// ---------------------------------------------------------------------------------------
struct Recycler {
    std::mutex mu;
    std::vector<std::pair<int, hipEvent_t>> events;
    std::vector<std::pair<int, hipStream_t>> streams;
};
inline Recycler& recycler() {
    static Recycler* r = new Recycler();  // never destroyed: in use until process exit
    return *r;
}
inline hipError_t take_event(hipEvent_t* e) {
    int dev = 0;
    hipError_t err = hipGetDevice(&dev);
    if (err != hipSuccess) return err;
    {
        Recycler& r = recycler();
        std::lock_guard<std::mutex> lk(r.mu);
        for (size_t i = 0; i < r.events.size(); ++i)
            if (r.events[i].first == dev) {
                *e = r.events[i].second;
                r.events[i] = r.events.back();
                r.events.pop_back();
                return hipSuccess;
            }
    }
    return hipEventCreateWithFlags(e, hipEventDisableTiming);
}
inline void give_event(hipEvent_t e, int dev) {
    if (!e) return;
    Recycler& r = recycler();
    std::lock_guard<std::mutex> lk(r.mu);
    r.events.emplace_back(dev, e);
}
inline hipError_t take_stream(hipStream_t* s) {
    int dev = 0;
    hipError_t err = hipGetDevice(&dev);
    if (err != hipSuccess) return err;
    {
        Recycler& r = recycler();
        std::lock_guard<std::mutex> lk(r.mu);
        for (size_t i = 0; i < r.streams.size(); ++i)
            if (r.streams[i].first == dev) {
                *s = r.streams[i].second;
                r.streams[i] = r.streams.back();
                r.streams.pop_back();
                return hipSuccess;
            }
    }
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}
inline void give_stream(hipStream_t s, int dev) {
    if (!s) return;
    Recycler& r = recycler();
    std::lock_guard<std::mutex> lk(r.mu);
    r.streams.emplace_back(dev, s);
}

// ---------------------------------------------------------------------------------------
// Loopback communicator: N simulated ranks of ONE process (one host thread per rank, all
// on the current GPU).  It lets the world > 1 code of the sharded step — gathered-chunk
// offsets, all-to-all splits, the side-stream event pipeline — run unchanged without N
// GPUs: every collective is a host rendezvous of the N callers, after which each rank
// enqueues device copies from its peers' posted buffers on its own stream, ordered after
// the peers' producers by events, and its stream is ordered after every copy that reads
// its own send buffers (RCCL's completion semantics: a collective is done on a rank's
// stream once its send buffers may be reused).
// ---------------------------------------------------------------------------------------
struct LoopPost {                 // what one rank posts for one collective
    std::vector<const char*> send;  // per peer: the bytes this rank sends to it
    std::vector<size_t> sbytes;
    std::vector<char*> recv;        // per peer: where this rank receives from it
    std::vector<size_t> rbytes;
};

struct LoopGroup {
    int n = 0, live = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    std::vector<LoopPost> post;
    std::vector<hipEvent_t> ready, done;  // per rank: its sends produced / its copies done
    int device = 0;                       // where the events were made
    int err = 0;                          // first failure of the current collective

    bool broken = false;                  // a rank gave up waiting: the group is unusable

    // generation barrier over the n ranks (host threads); false if a rank has not arrived
    // within 120 s (a rank that failed before the collective never will)
    bool barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (broken) return false;
        const uint64_t g = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return gen != g || broken; }) ||
            broken) {
            broken = true;
            cv.notify_all();
            return false;
        }
        return true;
    }
};

struct LoopComm {
    LoopGroup* g;
    int rank;
    bool exchange_failed = false;  // the last failure of this rank came from loop_exchange
    int exchanges_left = 0;        // collectives of the current step not yet joined
};

// A rank that fails before it joins a collective never arrives: mark the group broken and
// wake its peers, which then return an error at once instead of after the 120 s timeout.
static void loop_abort(LoopComm* c) {
    std::lock_guard<std::mutex> lk(c->g->mu);
    c->g->broken = true;
    c->g->cv.notify_all();
}

static std::mutex g_loop_mu;
static std::set<const void*> g_loop_comms;  // handles made by et_comm_loopback

static LoopComm* as_loop(const void* comm) {
    std::lock_guard<std::mutex> lk(g_loop_mu);
    return g_loop_comms.count(comm) ? (LoopComm*)comm : nullptr;
}

// One loopback exchange: rank r sends send[p] (sbytes[p]) to every peer p and receives
// recv[p] (rbytes[p]) from it.  Collective over the group's ranks; stream-ordered on st.
static int loop_exchange_impl(LoopComm* c, LoopPost&& mine, hipStream_t st);
static int loop_exchange(LoopComm* c, LoopPost&& mine, hipStream_t st) {
    if (c->exchanges_left > 0) --c->exchanges_left;
    const int rc = loop_exchange_impl(c, std::move(mine), st);
    c->exchange_failed = rc != ET_OK;
    return rc;
}

static int loop_exchange_impl(LoopComm* c, LoopPost&& mine, hipStream_t st) {
    LoopGroup& g = *c->g;
    const int r = c->rank;
    hipError_t e = hipEventRecord(g.ready[r], st);
    g.post[r] = std::move(mine);
    if (e != hipSuccess) {
        std::lock_guard<std::mutex> lk(g.mu);
        g.err = ET_ERR_HIP;
    }
    if (!g.barrier())  // every rank's buffers and events are posted
        return fail(ET_ERR_ARG, "loopback exchange: a rank did not join the collective");
    int bad = 0;
    {
        std::lock_guard<std::mutex> lk(g.mu);
        bad = g.err;
        for (int p = 0; p < g.n && !bad; ++p)
            if (g.post[p].sbytes.size() != (size_t)g.n || g.post[r].rbytes[p] != g.post[p].sbytes[r])
                bad = ET_ERR_ARG;
    }
    for (int p = 0; p < g.n && !bad && e == hipSuccess; ++p) {
        const size_t nb = g.post[r].rbytes[p];
        if (!nb) continue;
        if (p != r) e = hipStreamWaitEvent(st, g.ready[p], 0);
        if (e == hipSuccess)
            e = hipMemcpyAsync(g.post[r].recv[p], g.post[p].send[r], nb, hipMemcpyDeviceToDevice, st);
    }
    if (e == hipSuccess) e = hipEventRecord(g.done[r], st);
    if (e != hipSuccess && !bad) {
        std::lock_guard<std::mutex> lk(g.mu);
        g.err = ET_ERR_HIP;
    }
    if (!g.barrier())  // every rank's copies are enqueued
        return fail(ET_ERR_ARG, "loopback exchange: a rank did not join the collective");
    for (int p = 0; p < g.n && !bad && e == hipSuccess; ++p)
        if (p != r) e = hipStreamWaitEvent(st, g.done[p], 0);
    {
        std::lock_guard<std::mutex> lk(g.mu);
        if (e != hipSuccess && !g.err) g.err = ET_ERR_HIP;
        bad = bad ? bad : g.err;
    }
    // everyone has read err; then the next collective starts clean
    if (!g.barrier()) return fail(ET_ERR_ARG, "loopback exchange: a rank did not join the collective");
    if (r == 0) {
        std::lock_guard<std::mutex> lk(g.mu);
        g.err = 0;
    }
    if (!g.barrier()) return fail(ET_ERR_ARG, "loopback exchange: a rank did not join the collective");
    if (bad == ET_ERR_ARG) return fail(ET_ERR_ARG, "loopback exchange: the ranks' send and receive sizes differ");
    if (bad) return fail(ET_ERR_HIP, "loopback exchange: a HIP call failed on some rank");
    return ET_OK;
}

static LoopPost loop_allgather_post(int n, int rank, const void* send, void* recv, size_t bytes) {
    LoopPost m;
    m.send.assign(n, (const char*)send);
    m.sbytes.assign(n, bytes);
    m.recv.resize(n);
    m.rbytes.assign(n, bytes);
    for (int p = 0; p < n; ++p) m.recv[p] = (char*)recv + size_t(p) * bytes;
    (void)rank;
    return m;
}

// Grouped point-to-point exchange over RCCL: rank sends send[p] to p and receives recv[p]
// from p.  A failure inside the group still closes it (a group left open breaks every
// later RCCL call of the thread).
static int nccl_exchange(ncclComm_t comm, const LoopPost& m, hipStream_t st) {
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) return fail(ET_ERR_HIP, "ncclGroupStart failed: %s", ncclGetErrorString(r));
    const int n = (int)m.send.size();
    for (int p = 0; p < n && r == ncclSuccess; ++p) {
        if (m.sbytes[p]) r = ncclSend(m.send[p], m.sbytes[p], ncclUint8, p, comm, st);
        if (r == ncclSuccess && m.rbytes[p]) r = ncclRecv(m.recv[p], m.rbytes[p], ncclUint8, p, comm, st);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess) return fail(ET_ERR_HIP, "ncclSend/ncclRecv failed: %s", ncclGetErrorString(r));
    if (r2 != ncclSuccess) return fail(ET_ERR_HIP, "ncclGroupEnd failed: %s", ncclGetErrorString(r2));
    return ET_OK;
}

static const int kPieceDims[] = {512, 256, 128, 64, 32, 16};  // vector-kernel feature widths

static bool is_vec_dim(int d) {
    for (int v : kPieceDims)
        if (v == d) return true;
    return false;
}

// A feature range of one table cut into vector-kernel widths where alignment allows
// (96 -> 64 + 32); anything else stays one piece (the generic kernel takes it).
static void vec_split(int rank, int t, int f0, int dim, int64_t col, int es,
                      std::vector<et_shard_piece>& out) {
    while (dim > 0) {
        int w = 0;
        if ((int64_t(f0) * es) % 16 == 0)
            for (int v : kPieceDims)
                if (v <= dim) { w = v; break; }
        if (w == 0 || (!is_vec_dim(dim) && dim % 16 != 0)) {
            out.push_back({rank, t, f0, dim, col});
            return;
        }
        out.push_back({rank, t, f0, w, col});
        f0 += w;
        dim -= w;
        col += w;
    }
}

// Whole tables balanced by COUNT over the ranks, contiguous groups; with sizes, the
// tables are dealt in descending size round-robin (the largest on distinct ranks).
static std::vector<std::vector<int>> plan_tables(int ntables, int world, const int64_t* sizes) {
    int base = ntables / world, extra = ntables % world;
    std::vector<int> counts(world);
    for (int r = 0; r < world; ++r) counts[r] = base + (r < extra ? 1 : 0);
    std::vector<std::vector<int>> out(world);
    if (!sizes) {
        int t = 0;
        for (int r = 0; r < world; ++r)
            for (int c = 0; c < counts[r]; ++c) out[r].push_back(t++);
        return out;
    }
    std::vector<int> order(ntables);
    for (int t = 0; t < ntables; ++t) order[t] = t;
    std::stable_sort(order.begin(), order.end(),
                     [&](int a, int b) { return sizes[a] > sizes[b]; });
    int r = 0;
    for (int t : order) {
        while ((int)out[r].size() >= counts[r]) r = (r + 1) % world;
        out[r].push_back(t);
        r = (r + 1) % world;
    }
    for (auto& o : out) std::sort(o.begin(), o.end());
    return out;
}

// Cut points of the concatenated feature axis: table edges, and multiples of `granule`
// inside a table; each rank boundary is the candidate nearest an equal split.
static std::vector<int64_t> plan_features(int ntables, const int32_t* dims, int world,
                                          int granule) {
    std::set<int64_t> cuts{0};
    int64_t start = 0;
    for (int t = 0; t < ntables; ++t) {
        for (int64_t f = granule; f < dims[t]; f += granule) cuts.insert(start + f);
        start += dims[t];
        cuts.insert(start);
    }
    const int64_t F = start;
    std::vector<int64_t> bounds{0};
    for (int r = 1; r < world; ++r) {
        const double target = double(F) * r / world;
        int64_t best = -1;
        double bd = 0;
        for (int64_t c : cuts) {
            if (c < bounds.back()) continue;
            double d = std::fabs(double(c) - target);
            if (best < 0 || d < bd) { best = c; bd = d; }  // ties: the smaller cut (set order)
        }
        bounds.push_back(best);
    }
    bounds.push_back(F);
    return bounds;
}

// ---------------------------------------------------------------------------------------
// The sharded step
// ---------------------------------------------------------------------------------------
struct Launch {  // one et_concat_slabs / et_split_slabs launch of the assembly
    int64_t shift;
    std::vector<int32_t> rows;
    std::vector<int64_t> offs;
};

struct Sharded {
    ncclComm_t comm = nullptr;    // RCCL, or
    LoopComm* loop = nullptr;     // a loopback rank (et_comm_loopback)
    int world = 0, rank = 0, dtype = 0, es = 0, chunks = 1, exchange = 0, device = 0;
    int64_t prepend = 0, ld_dst = 0, batch = 0, slab_ld = 0;
    std::vector<std::vector<et_shard_piece>> pieces;  // per rank, slab order
    std::vector<Launch> launches;
    std::vector<int64_t> bounds;  // batch chunk c = [bounds[c], bounds[c+1])
    std::vector<int64_t> split;   // all-to-all: rank j keeps batch rows [split[j], split[j+1])
    int64_t ws_slab = 0, ws_gathered = 0;
    hipStream_t side = nullptr;   // exchange + assembly stream
    std::vector<hipEvent_t> ev;   // per chunk: its lookup is done
    hipEvent_t ev_in = nullptr, ev_out = nullptr;
};

static int64_t round_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

static void build_launches(Sharded& s) {
    // contiguous (slab_col, dst_col, ncols) runs of each rank's slab
    std::vector<std::vector<std::array<int64_t, 3>>> runs(s.world);
    for (int r = 0; r < s.world; ++r) {
        int64_t sc = 0;
        for (auto& p : s.pieces[r]) {
            auto& rr = runs[r];
            if (!rr.empty() && rr.back()[0] + rr.back()[2] == sc && rr.back()[1] + rr.back()[2] == p.col)
                rr.back()[2] += p.dim;
            else
                rr.push_back({sc, p.col, p.dim});
            sc += p.dim;
        }
    }
    size_t kmax = 0;
    for (auto& r : runs) kmax = std::max(kmax, r.size());
    for (size_t k = 0; k < kmax; ++k) {
        std::map<int64_t, Launch> per;
        for (int r = 0; r < s.world; ++r) {
            if (k >= runs[r].size()) continue;
            auto& x = runs[r][k];
            Launch& L = per[x[0]];
            if (L.rows.empty()) {
                L.shift = x[0];
                L.rows.assign(s.world, 0);
                L.offs.assign(s.world, 0);
            }
            L.rows[r] = (int32_t)x[2];
            L.offs[r] = x[1];
        }
        for (auto& kv : per) s.launches.push_back(kv.second);
    }
}

static ncclDataType_t bytes_type() { return ncclUint8; }

// All-gather of one batch chunk of the slab, then its assembly into dst (on `st`).
static int exchange_chunk(Sharded& s, const char* slab_c, char* gath_c, int64_t nb, char* dst_c,
                          int64_t ld_dst, hipStream_t st) {
    const size_t bytes = size_t(nb) * s.slab_ld * s.es;
    if (s.loop) {
        int rc = loop_exchange(s.loop, loop_allgather_post(s.world, s.rank, slab_c, gath_c, bytes), st);
        if (rc != ET_OK) return rc;
    } else if (!s.comm) {
        ET_HIP_CHECK(hipMemcpyAsync(gath_c, slab_c, bytes, hipMemcpyDeviceToDevice, st));
    } else {
        ET_NCCL_CHECK(ncclAllGather(slab_c, gath_c, bytes, bytes_type(), s.comm, st));
    }
    for (auto& L : s.launches) {
        int rc = et_concat_slabs(s.dtype, gath_c + L.shift * s.es, s.world, s.slab_ld, nb,
                                 L.rows.data(), L.offs.data(), dst_c, ld_dst, st);
        if (rc != ET_OK) return rc;
    }
    return ET_OK;
}

static int lookup_chunk(Sharded& s, const et_lookup_desc* local, int32_t nlocal, int64_t b0,
                        int64_t b1, char* slab, uint32_t flags, hipStream_t st) {
    if (nlocal == 0 || b1 <= b0) return ET_OK;
    std::vector<et_lookup_desc> d(local, local + nlocal);
    int64_t off = 0;
    for (int i = 0; i < nlocal; ++i) {
        d[i].idx = local[i].idx + b0 * local[i].ld_idx;
        d[i].dst_row_off = off;
        off += local[i].dim;
    }
    return et_maplookup_prealloc(s.dtype, d.data(), nlocal, b1 - b0, slab + b0 * s.slab_ld * s.es,
                                 s.slab_ld, flags, st);
}

}  // namespace et

using et::Sharded;

extern "C" int et_shard_plan(int32_t mode, int32_t ntables, const int32_t* dims,
                             const int64_t* sizes, int32_t world, int64_t prependrows,
                             int32_t granule, int32_t elsize, et_shard_piece* out, int32_t cap,
                             int32_t* npieces) {
    et::clear_err();
    if (world <= 0) return et::fail(ET_ERR_ARG, "world must be positive");
    if (ntables < 0 || (ntables > 0 && !dims)) return et::fail(ET_ERR_ARG, "bad table list");
    if (mode != ET_PLAN_TABLEWISE && mode != ET_PLAN_FEATUREWISE)
        return et::fail(ET_ERR_ARG, "unknown plan mode %d", mode);
    if (mode == ET_PLAN_FEATUREWISE && (granule <= 0 || elsize <= 0))
        return et::fail(ET_ERR_ARG, "feature-wise plan needs granule > 0 and elsize > 0");
    for (int t = 0; t < ntables; ++t)
        if (dims[t] <= 0) return et::fail(ET_ERR_ARG, "table %d: dim %d", t, dims[t]);
    std::vector<int64_t> col(ntables);
    int64_t c = prependrows;
    for (int t = 0; t < ntables; ++t) { col[t] = c; c += dims[t]; }
    std::vector<et_shard_piece> v;
    if (mode == ET_PLAN_TABLEWISE) {
        auto ts = et::plan_tables(ntables, world, sizes);
        for (int r = 0; r < world; ++r)
            for (int t : ts[r]) v.push_back({r, t, 0, dims[t], col[t]});
    } else {
        auto b = et::plan_features(ntables, dims, world, granule);
        for (int r = 0; r < world; ++r)
            for (int t = 0; t < ntables; ++t) {
                int64_t st = col[t] - prependrows;
                int64_t lo = std::max(b[r], st), hi = std::min(b[r + 1], st + dims[t]);
                if (lo < hi)
                    et::vec_split(r, t, int(lo - st), int(hi - lo), prependrows + lo, elsize, v);
            }
    }
    if (npieces) *npieces = (int32_t)v.size();
    if (out) {
        if ((int64_t)v.size() > cap)
            return et::fail(ET_ERR_ARG, "plan has %zu pieces, output holds %d", v.size(), cap);
        std::copy(v.begin(), v.end(), out);
    }
    return ET_OK;
}

extern "C" int et_comm_unique_id(void* id) {
    et::clear_err();
    if (!id) return et::fail(ET_ERR_ARG, "id is NULL");
    ncclUniqueId u;
    ET_NCCL_CHECK(ncclGetUniqueId(&u));
    memcpy(id, &u, sizeof(u));
    return ET_OK;
}

extern "C" int et_comm_init(void** comm, int32_t nranks, const void* id, int32_t rank) {
    et::clear_err();
    if (!comm || !id || nranks <= 0 || rank < 0 || rank >= nranks)
        return et::fail(ET_ERR_ARG, "bad communicator arguments (nranks %d, rank %d)", nranks, rank);
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclComm_t c = nullptr;
    ET_NCCL_CHECK(ncclCommInitRank(&c, nranks, u, rank));
    *comm = c;
    return ET_OK;
}

extern "C" int et_comm_loopback(void** comms, int32_t nranks) {
    et::clear_err();
    if (!comms || nranks <= 0 || nranks > 1024)
        return et::fail(ET_ERR_ARG, "bad loopback arguments (nranks %d)", nranks);
    et::LoopGroup* g = new (std::nothrow) et::LoopGroup();
    if (!g) return et::fail(ET_ERR_ARG, "out of host memory");
    g->n = g->live = nranks;
    g->post.resize(nranks);
    g->ready.assign(nranks, nullptr);
    g->done.assign(nranks, nullptr);
    hipError_t e = hipGetDevice(&g->device);
    for (int r = 0; r < nranks && e == hipSuccess; ++r) {
        e = et::take_event(&g->ready[r]);
        if (e == hipSuccess) e = et::take_event(&g->done[r]);
    }
    if (e != hipSuccess) {
        for (int r = 0; r < nranks; ++r) {
            et::give_event(g->ready[r], g->device);
            et::give_event(g->done[r], g->device);
        }
        delete g;
        return et::fail(ET_ERR_HIP, "event creation failed: %s", hipGetErrorString(e));
    }
    std::lock_guard<std::mutex> lk(et::g_loop_mu);
    for (int r = 0; r < nranks; ++r) {
        comms[r] = new et::LoopComm{g, r};
        et::g_loop_comms.insert(comms[r]);
    }
    return ET_OK;
}

extern "C" int et_comm_destroy(void* comm) {
    et::clear_err();
    if (!comm) return ET_OK;
    {
        std::lock_guard<std::mutex> lk(et::g_loop_mu);
        if (et::g_loop_comms.erase(comm)) {
            et::LoopComm* c = (et::LoopComm*)comm;
            et::LoopGroup* g = c->g;
            delete c;
            if (--g->live == 0) {  // the last rank of the group frees it (events recycled)
                for (int r = 0; r < g->n; ++r) {
                    et::give_event(g->ready[r], g->device);
                    et::give_event(g->done[r], g->device);
                }
                delete g;
            }
            return ET_OK;
        }
    }
    ET_NCCL_CHECK(ncclCommDestroy((ncclComm_t)comm));
    return ET_OK;
}

extern "C" int et_allgather_concat(void* comm, int dtype, const void* slab, int64_t slab_ld,
                                   int64_t batch, void* gathered, int32_t nranks,
                                   const int32_t* rows, const int64_t* dst_row_off, void* dst,
                                   int64_t ld_dst, void* stream) {
    et::clear_err();
    const int es = et::elsize(dtype);
    if (!es) return et::fail(ET_ERR_ARG, "unknown dtype %d", dtype);
    if (nranks <= 0 || slab_ld <= 0 || batch < 0 || !rows || !dst_row_off)
        return et::fail(ET_ERR_ARG, "bad all-gather arguments");
    if (nranks > 1 && !comm) return et::fail(ET_ERR_ARG, "communicator is NULL");
    if (batch == 0) return ET_OK;
    hipStream_t st = (hipStream_t)stream;
    const size_t bytes = size_t(batch) * slab_ld * es;
    if (et::LoopComm* lc = et::as_loop(comm)) {
        if (lc->g->n != nranks) return et::fail(ET_ERR_ARG, "loopback group of %d ranks, nranks %d", lc->g->n, nranks);
        int rc = et::loop_exchange(lc, et::loop_allgather_post(nranks, lc->rank, slab, gathered, bytes), st);
        if (rc != ET_OK) return rc;
    } else if (!comm) {
        ET_HIP_CHECK(hipMemcpyAsync(gathered, slab, bytes, hipMemcpyDeviceToDevice, st));
    } else {
        ET_NCCL_CHECK(ncclAllGather(slab, gathered, bytes, ncclUint8, (ncclComm_t)comm, st));
    }
    return et_concat_slabs(dtype, gathered, nranks, slab_ld, batch, rows, dst_row_off, dst, ld_dst,
                           stream);
}

extern "C" int et_sharded_create(void** handle, void* comm, int32_t world, int32_t rank,
                                 int dtype, const et_shard_piece* pieces, int32_t npieces,
                                 int64_t prependrows, int64_t ld_dst, int64_t batch,
                                 int32_t chunks, int32_t exchange) {
    et::clear_err();
    if (!handle) return et::fail(ET_ERR_ARG, "handle is NULL");
    *handle = nullptr;
    const int es = et::elsize(dtype);
    if (!es) return et::fail(ET_ERR_ARG, "unknown dtype %d", dtype);
    if (world <= 0 || rank < 0 || rank >= world)
        return et::fail(ET_ERR_ARG, "rank %d of world %d", rank, world);
    if (world > 1 && !comm) return et::fail(ET_ERR_ARG, "world %d needs a communicator", world);
    if (exchange != ET_EXCHANGE_ALLGATHER && exchange != ET_EXCHANGE_ALLTOALL)
        return et::fail(ET_ERR_ARG, "unknown exchange %d", exchange);
    if (batch <= 0 || npieces < 0 || (npieces > 0 && !pieces))
        return et::fail(ET_ERR_ARG, "bad batch / piece list");
    Sharded* s = new (std::nothrow) Sharded();
    if (!s) return et::fail(ET_ERR_ARG, "out of host memory");
    s->loop = et::as_loop(comm);
    s->comm = s->loop ? nullptr : (ncclComm_t)comm;
    if (s->loop && (s->loop->g->n != world || s->loop->rank != rank)) {
        delete s;
        return et::fail(ET_ERR_ARG, "loopback communicator is rank %d of %d, not %d of %d",
                        ((et::LoopComm*)comm)->rank, ((et::LoopComm*)comm)->g->n, rank, world);
    }
    s->world = world;
    s->rank = rank;
    s->dtype = dtype;
    s->es = es;
    s->exchange = exchange;
    s->prepend = prependrows;
    s->ld_dst = ld_dst;
    s->batch = batch;
    s->pieces.assign(world, {});
    int64_t maxw = 0;
    for (int i = 0; i < npieces; ++i) {
        const et_shard_piece& p = pieces[i];
        if (p.rank < 0 || p.rank >= world || p.dim <= 0 || p.col < prependrows ||
            p.col + p.dim > ld_dst) {
            delete s;
            return et::fail(ET_ERR_ARG, "piece %d (rank %d, dim %d, col %lld) outside the plan",
                            i, p.rank, p.dim, (long long)p.col);
        }
        s->pieces[p.rank].push_back(p);
    }
    for (auto& v : s->pieces) {
        int64_t w = 0;
        for (auto& p : v) w += p.dim;
        maxw = std::max(maxw, w);
    }
    // equal slabs for the collective; a multiple of 16 bytes keeps vector stores aligned
    s->slab_ld = std::max<int64_t>(16 / es, et::round_up(maxw, std::max(1, 16 / es)));
    s->chunks = exchange == ET_EXCHANGE_ALLTOALL ? 1 : (int)std::max<int64_t>(1, std::min<int64_t>(chunks, batch));
    for (int c = 0; c <= s->chunks; ++c) s->bounds.push_back(batch * c / s->chunks);
    for (int j = 0; j <= world; ++j) s->split.push_back(batch * j / world);
    et::build_launches(*s);
    const int64_t mine = s->split[rank + 1] - s->split[rank];
    s->ws_slab = et::round_up(batch * s->slab_ld * es, 256);
    s->ws_gathered = et::round_up(int64_t(world) *
                                      (exchange == ET_EXCHANGE_ALLTOALL ? mine : batch) *
                                      s->slab_ld * es, 256);
    hipError_t e = hipGetDevice(&s->device);
    if (e == hipSuccess && s->chunks > 1) {
        e = et::take_stream(&s->side);
        s->ev.assign(s->chunks, nullptr);
        for (int c = 0; e == hipSuccess && c < s->chunks; ++c) e = et::take_event(&s->ev[c]);
        if (e == hipSuccess) e = et::take_event(&s->ev_in);
        if (e == hipSuccess) e = et::take_event(&s->ev_out);
    }
    if (e != hipSuccess) {
        et_sharded_destroy(s);
        return et::fail(ET_ERR_HIP, "stream / event creation failed: %s", hipGetErrorString(e));
    }
    *handle = s;
    return ET_OK;
}

extern "C" int et_sharded_info(void* handle, int64_t* slab_ld, int64_t* ws_bytes,
                               int64_t* batch_lo, int64_t* batch_hi) {
    et::clear_err();
    if (!handle) return et::fail(ET_ERR_ARG, "handle is NULL");
    Sharded* s = (Sharded*)handle;
    if (slab_ld) *slab_ld = s->slab_ld;
    if (ws_bytes) *ws_bytes = s->ws_slab + s->ws_gathered;
    if (batch_lo) *batch_lo = s->exchange == ET_EXCHANGE_ALLTOALL ? s->split[s->rank] : 0;
    if (batch_hi) *batch_hi = s->exchange == ET_EXCHANGE_ALLTOALL ? s->split[s->rank + 1] : s->batch;
    return ET_OK;
}

static int check_local(Sharded* s, const et_lookup_desc* local, int32_t nlocal) {
    const auto& mine = s->pieces[s->rank];
    if (nlocal != (int32_t)mine.size())
        return et::fail(ET_ERR_ARG, "rank %d owns %zu pieces, %d descriptors given", s->rank,
                        mine.size(), nlocal);
    for (int i = 0; i < nlocal; ++i)
        if (local[i].dim != mine[i].dim)
            return et::fail(ET_ERR_ARG, "descriptor %d: dim %d, piece dim %d", i, local[i].dim,
                            mine[i].dim);
    return ET_OK;
}

// A loopback rank whose step fails outside a collective (argument checks, a lookup launch)
// BEFORE it has joined every collective of the step aborts its group, so its peers' pending
// collectives fail fast.  A failure after its last collective (an assembly
// launch) leaves the group alone: its peers' step completed.
static int loop_guard(Sharded* s, int rc) {
    if (rc != ET_OK && s->loop && !s->loop->exchange_failed && s->loop->exchanges_left > 0)
        et::loop_abort(s->loop);
    if (s->loop) s->loop->exchanges_left = 0;
    return rc;
}

static int sharded_maplookup(Sharded* s, const et_lookup_desc* local, int32_t nlocal, void* dst,
                             int64_t ld_dst, void* workspace, int64_t ws_bytes, uint32_t flags,
                             void* stream);
static int sharded_piece_grads(Sharded* s, const void* delta, int64_t ld_delta, void* recv,
                               void* workspace, int64_t ws_bytes, void* stream);

extern "C" int et_sharded_maplookup(void* handle, const et_lookup_desc* local, int32_t nlocal,
                                    void* dst, int64_t ld_dst, void* workspace, int64_t ws_bytes,
                                    uint32_t flags, void* stream) {
    et::clear_err();
    if (!handle) return et::fail(ET_ERR_ARG, "handle is NULL");
    Sharded* s = (Sharded*)handle;
    if (s->loop) {
        s->loop->exchange_failed = false;
        s->loop->exchanges_left = s->exchange == ET_EXCHANGE_ALLTOALL ? 1 : s->chunks;
    }
    return loop_guard(s, sharded_maplookup(s, local, nlocal, dst, ld_dst, workspace, ws_bytes,
                                           flags, stream));
}

extern "C" int et_sharded_piece_grads(void* handle, const void* delta, int64_t ld_delta,
                                      void* recv, void* workspace, int64_t ws_bytes,
                                      void* stream) {
    et::clear_err();
    if (!handle) return et::fail(ET_ERR_ARG, "handle is NULL");
    Sharded* s = (Sharded*)handle;
    if (s->loop) {
        s->loop->exchange_failed = false;
        s->loop->exchanges_left = 1;
    }
    return loop_guard(s, sharded_piece_grads(s, delta, ld_delta, recv, workspace, ws_bytes,
                                             stream));
}

static int sharded_maplookup(Sharded* s, const et_lookup_desc* local, int32_t nlocal, void* dst,
                             int64_t ld_dst, void* workspace, int64_t ws_bytes, uint32_t flags,
                             void* stream) {
    int rc = check_local(s, local, nlocal);
    if (rc != ET_OK) return rc;
    if (ld_dst < s->ld_dst) return et::fail(ET_ERR_ARG, "ld_dst %lld < plan's %lld", (long long)ld_dst, (long long)s->ld_dst);
    if (!workspace || ws_bytes < s->ws_slab + s->ws_gathered)
        return et::fail(ET_ERR_WORKSPACE, "workspace of %lld bytes, %lld needed", (long long)ws_bytes,
                        (long long)(s->ws_slab + s->ws_gathered));
    hipStream_t st = (hipStream_t)stream;
    char* slab = (char*)workspace;
    char* gath = slab + s->ws_slab;
    char* d = (char*)dst;
    const int64_t row = s->slab_ld * s->es;
    if (s->exchange == ET_EXCHANGE_ALLTOALL) {
        // DLRM layout: rank j keeps batch rows [split[j], split[j+1]) of every rank's slab
        if ((rc = et::lookup_chunk(*s, local, nlocal, 0, s->batch, slab, flags, st)) != ET_OK) return rc;
        const int64_t mine = s->split[s->rank + 1] - s->split[s->rank];
        if (!s->comm && !s->loop) {
            ET_HIP_CHECK(hipMemcpyAsync(gath, slab, size_t(mine) * row, hipMemcpyDeviceToDevice, st));
        } else {
            // rank p gets bags [split[p], split[p+1]) of this slab; this rank receives its
            // own bag slice of every rank's slab, rank after rank
            et::LoopPost m;
            for (int p = 0; p < s->world; ++p) {
                const int64_t n = s->split[p + 1] - s->split[p];
                m.send.push_back(slab + s->split[p] * row);
                m.sbytes.push_back(size_t(n) * row);
                m.recv.push_back(gath + p * mine * row);
                m.rbytes.push_back(size_t(mine) * row);
            }
            rc = s->loop ? et::loop_exchange(s->loop, std::move(m), st) : et::nccl_exchange(s->comm, m, st);
            if (rc != ET_OK) return rc;
        }
        for (auto& L : s->launches)
            if ((rc = et_concat_slabs(s->dtype, gath + L.shift * s->es, s->world, s->slab_ld, mine,
                                      L.rows.data(), L.offs.data(), d, ld_dst, st)) != ET_OK)
                return rc;
        return ET_OK;
    }
    if (s->chunks == 1) {
        if ((rc = et::lookup_chunk(*s, local, nlocal, 0, s->batch, slab, flags, st)) != ET_OK) return rc;
        return et::exchange_chunk(*s, slab, gath, s->batch, d, ld_dst, st);
    }
    // pipelined: chunk c+1's lookup on the caller's stream while chunk c is exchanged and
    // assembled on the side stream (the previous step's users of dst / slab came first)
    ET_HIP_CHECK(hipEventRecord(s->ev_in, st));
    ET_HIP_CHECK(hipStreamWaitEvent(s->side, s->ev_in, 0));
    for (int c = 0; c < s->chunks; ++c) {
        const int64_t b0 = s->bounds[c], b1 = s->bounds[c + 1];
        if ((rc = et::lookup_chunk(*s, local, nlocal, b0, b1, slab, flags, st)) != ET_OK) return rc;
        ET_HIP_CHECK(hipEventRecord(s->ev[c], st));
        ET_HIP_CHECK(hipStreamWaitEvent(s->side, s->ev[c], 0));
        if ((rc = et::exchange_chunk(*s, slab + b0 * row, gath + s->world * b0 * row, b1 - b0,
                                     d + b0 * ld_dst * s->es, ld_dst, s->side)) != ET_OK)
            return rc;
    }
    ET_HIP_CHECK(hipEventRecord(s->ev_out, s->side));
    ET_HIP_CHECK(hipStreamWaitEvent(st, s->ev_out, 0));
    return ET_OK;
}

static int sharded_piece_grads(Sharded* s, const void* delta, int64_t ld_delta, void* recv,
                               void* workspace, int64_t ws_bytes, void* stream) {
    if (s->exchange != ET_EXCHANGE_ALLTOALL)
        return et::fail(ET_ERR_ARG, "all-gather layout: a piece's gradient is a column view of "
                                    "the replicated gradient (no exchange)");
    if (!workspace || ws_bytes < s->ws_slab + s->ws_gathered)
        return et::fail(ET_ERR_WORKSPACE, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    const int64_t row = s->slab_ld * s->es;
    const int64_t mine = s->split[s->rank + 1] - s->split[s->rank];
    char* send = (char*)workspace + s->ws_slab;  // world x mine x slab_ld
    int rc;
    ET_HIP_CHECK(hipMemsetAsync(send, 0, size_t(s->world) * mine * row, st));
    for (auto& L : s->launches)
        if ((rc = et_split_slabs(s->dtype, delta, ld_delta, mine, s->world, L.rows.data(),
                                 L.offs.data(), send + L.shift * s->es, s->slab_ld, st)) != ET_OK)
            return rc;
    char* out = (char*)recv;  // batch x slab_ld: every bag, this rank's features
    if (!s->comm && !s->loop) {
        ET_HIP_CHECK(hipMemcpyAsync(out, send, size_t(mine) * row, hipMemcpyDeviceToDevice, st));
        return ET_OK;
    }
    et::LoopPost m;
    for (int p = 0; p < s->world; ++p) {
        const int64_t n = s->split[p + 1] - s->split[p];
        m.send.push_back(send + p * mine * row);
        m.sbytes.push_back(size_t(mine) * row);
        m.recv.push_back(out + s->split[p] * row);
        m.rbytes.push_back(size_t(n) * row);
    }
    return s->loop ? et::loop_exchange(s->loop, std::move(m), st) : et::nccl_exchange(s->comm, m, st);
}

extern "C" int et_sharded_destroy(void* handle) {
    et::clear_err();
    Sharded* s = (Sharded*)handle;
    if (!s) return ET_OK;
    int dev = -1;
    if (hipGetDevice(&dev) == hipSuccess && dev != s->device) (void)hipSetDevice(s->device);
    // recycled, not destroyed (see Recycler): callers' streams may have waited on them
    for (hipEvent_t e : s->ev) et::give_event(e, s->device);
    et::give_event(s->ev_in, s->device);
    et::give_event(s->ev_out, s->device);
    et::give_stream(s->side, s->device);
    if (dev >= 0 && dev != s->device) (void)hipSetDevice(dev);
    delete s;
    return ET_OK;
}
