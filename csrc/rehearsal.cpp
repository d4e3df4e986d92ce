// Asynchronous rehearsal collectives (scaling_amd/core/topology/gloo_gpu.py, SCALING_AMD_REHEARSAL_ASYNC=1): the
// worker that runs every gloo call of a rank in program order, in C++ so that it never needs the Python GIL.
//
// The Python side enqueues, on the collective's HIP stream, the input's device-to-host copy into pinned memory, an
// event, a stream gate (hipStreamWaitValue32 on a flag word) and the result's host-to-device copy, then hands this
// worker a job: wait for the event (the stream has copied the input out), run the collective on the host tensors with
// the group's c10d ProcessGroup (gloo), write the result and open the gate.  A Python thread doing this would need
// the GIL between those steps -- and a main thread blocked in a GIL-holding call (a .tolist() of a tensor behind the
// gate) then deadlocks the rank.  Python-level gloo calls (CPU tensors, object collectives, barriers) are serialised
// with the queued jobs through host_begin / host_end: the main thread waits (GIL released) until the worker reaches
// its turn, runs the call itself, and lets the worker go on.
#include <torch/extension.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>

#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>

namespace {

const bool kTrace = [] {
    const char* e = std::getenv("SCALING_AMD_REHEARSAL_TRACE");
    return e != nullptr && e[0] == '1';
}();
void trace(const char* what, int64_t idx, int64_t kind) {
    if (!kTrace) return;
    const char* r = std::getenv("RANK");
    std::fprintf(stderr, "[rehearsal worker r%s] %s job gate %lld kind %lld\n", r ? r : "?", what, (long long)idx,
                 (long long)kind);
}

struct Worker {
    std::mutex m;
    std::condition_variable cv;
    std::deque<std::function<void()>> q;
    std::thread t;
    std::string error;
    // host_begin / host_end hand-over
    int64_t host_turn = -1, host_next = 0;
    bool host_running = false;

    Worker() { t = std::thread([this] { loop(); }); t.detach(); }
    void loop() {
        for (;;) {
            std::function<void()> job;
            {
                std::unique_lock<std::mutex> lk(m);
                cv.wait(lk, [this] { return !q.empty(); });
                job = std::move(q.front());
                q.pop_front();
            }
            job();
        }
    }
    void push(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> lk(m);
            q.push_back(std::move(f));
        }
        cv.notify_all();
    }
};

Worker& worker() {
    static Worker* w = new Worker();  // lives for the process (the detached thread may outlive static destruction)
    return *w;
}

void fail(const std::string& what) {
    Worker& w = worker();
    std::lock_guard<std::mutex> lk(w.m);
    if (w.error.empty()) w.error = what;
}

void open_gate(int64_t base, int64_t idx, int64_t gen) {
    std::atomic_thread_fence(std::memory_order_seq_cst);
    __atomic_store_n(reinterpret_cast<uint32_t*>((uintptr_t)base) + idx, (uint32_t)gen, __ATOMIC_SEQ_CST);
}

c10d::ReduceOp red_op(int64_t op) {
    switch (op) {
        case 1: return c10d::ReduceOp(c10d::ReduceOp::MAX);
        case 2: return c10d::ReduceOp(c10d::ReduceOp::MIN);
        case 3: return c10d::ReduceOp(c10d::ReduceOp::PRODUCT);
        default: return c10d::ReduceOp(c10d::ReduceOp::SUM);
    }
}

// SUM over the group in rank order (gloo sums 3+ ranks in message-arrival order; RCCL's ring order is fixed)
at::Tensor ordered_sum(const c10::intrusive_ptr<c10d::ProcessGroup>& pg, const at::Tensor& h) {
    const int n = pg->getSize();
    at::Tensor flat = h.contiguous().reshape({-1});
    at::Tensor parts = at::empty({n * flat.numel()}, flat.options());
    pg->_allgather_base(parts, flat)->wait();
    parts = parts.view({n, -1});
    at::Tensor out = parts[0].clone();
    for (int i = 1; i < n; ++i) out.add_(parts[i]);
    return out.view(h.sizes());
}

// kind: 0 all_reduce (in place on h_in == h_out), 1 broadcast (in place; root = group rank), 2 reduce_scatter
// (h_in full, h_out this rank's slice), 3 all_gather_into (h_in shard, h_out full)
void run(int64_t kind, const c10::intrusive_ptr<c10d::ProcessGroup>& pg, at::Tensor h_in, at::Tensor h_out, int64_t op,
         int64_t root) {
    const int n = pg->getSize();
    const bool ordered = op == 0 && n > 2;
    if (kind == 0) {
        if (ordered) {
            h_out.copy_(ordered_sum(pg, h_in));
        } else {
            std::vector<at::Tensor> v{h_in};
            c10d::AllreduceOptions o;
            o.reduceOp = red_op(op);
            pg->allreduce(v, o)->wait();
            if (!h_out.is_same(h_in)) h_out.copy_(h_in);
        }
    } else if (kind == 1) {
        std::vector<at::Tensor> v{h_in};
        c10d::BroadcastOptions o;
        o.rootRank = root;
        pg->broadcast(v, o)->wait();
        if (!h_out.is_same(h_in)) h_out.copy_(h_in);
    } else if (kind == 2) {
        if (ordered) {
            const int64_t k = h_out.numel(), r = pg->getRank();
            h_out.copy_(ordered_sum(pg, h_in).reshape({-1}).slice(0, r * k, (r + 1) * k).view(h_out.sizes()));
        } else {
            c10d::ReduceScatterOptions o;
            o.reduceOp = red_op(op);
            pg->_reduce_scatter_base(h_out, h_in, o)->wait();
        }
    } else {
        pg->_allgather_base(h_out, h_in)->wait();
    }
}

}  // namespace

// Queue one collective: the job waits for `event` (a hipEvent_t recorded after the input's copy-out), runs the
// collective on the pinned host tensors and opens gate (base, idx) at generation `gen` -- also when it fails (the
// stream must not wait forever; the error is raised by the next rw_check).
void rw_collective(int64_t kind, const c10::intrusive_ptr<c10d::ProcessGroup>& pg, at::Tensor h_in, at::Tensor h_out,
                   int64_t op, int64_t root, int64_t event, int64_t base, int64_t idx, int64_t gen) {
    worker().push([=]() {
        trace("start", idx, kind);
        try {
            if (event != 0)  // 0: host-only job (the CPU tests of the worker)
                TORCH_CHECK(hipEventSynchronize(reinterpret_cast<hipEvent_t>((uintptr_t)event)) == hipSuccess,
                            "rehearsal worker: hipEventSynchronize");
            trace("input out", idx, kind);
            run(kind, pg, h_in, h_out, op, root);
            trace("collective done", idx, kind);
        } catch (const std::exception& e) {
            fail(e.what());
        } catch (...) {
            fail("rehearsal worker: unknown error");
        }
        open_gate(base, idx, gen);
    });
}

// Pipeline p2p (the framework's batched isend / irecv).  A send job waits for `event` (the payload's copy-out),
// POSTS the gloo sends and returns without waiting for them (a send completes when the peer receives, which may be a
// later job of the peer's worker -- as an RCCL send runs on its own stream); their works are kept under `send_id` for
// rw_send_wait.  A receive job posts its receives, waits for them, and opens gate (base, idx) at `gen`.
// peers are group ranks of `pg`.
static std::mutex g_sends_m;
static std::map<int64_t, std::vector<c10::intrusive_ptr<c10d::Work>>> g_sends;

void rw_p2p_send(const c10::intrusive_ptr<c10d::ProcessGroup>& pg, std::vector<at::Tensor> hs, std::vector<int64_t> peers,
                 std::vector<int64_t> tags, int64_t event, int64_t send_id) {
    worker().push([=]() {
        trace("start send", send_id, 4);
        try {
            if (event != 0)
                TORCH_CHECK(hipEventSynchronize(reinterpret_cast<hipEvent_t>((uintptr_t)event)) == hipSuccess,
                            "rehearsal worker: hipEventSynchronize");
            std::vector<c10::intrusive_ptr<c10d::Work>> works;
            for (size_t i = 0; i < hs.size(); ++i) {
                std::vector<at::Tensor> v{hs[i]};
                works.push_back(pg->send(v, (int)peers[i], (int)tags[i]));
            }
            std::lock_guard<std::mutex> lk(g_sends_m);
            g_sends[send_id] = std::move(works);
        } catch (const std::exception& e) {
            fail(e.what());
        } catch (...) {
            fail("rehearsal worker: unknown error");
        }
        trace("sends posted", send_id, 4);
    });
}

void rw_p2p_recv(const c10::intrusive_ptr<c10d::ProcessGroup>& pg, std::vector<at::Tensor> hs, std::vector<int64_t> peers,
                 std::vector<int64_t> tags, int64_t base, int64_t idx, int64_t gen) {
    worker().push([=]() {
        trace("start recv", idx, 5);
        try {
            std::vector<c10::intrusive_ptr<c10d::Work>> works;
            for (size_t i = 0; i < hs.size(); ++i) {
                std::vector<at::Tensor> v{hs[i]};
                works.push_back(pg->recv(v, (int)peers[i], (int)tags[i]));
            }
            for (auto& w : works) w->wait();
        } catch (const std::exception& e) {
            fail(e.what());
        } catch (...) {
            fail("rehearsal worker: unknown error");
        }
        trace("received", idx, 5);
        open_gate(base, idx, gen);
    });
}

// Waits (GIL released) until the sends of `send_id` have completed, in program order (called inside a host turn, so
// the worker has posted them).
void rw_send_wait(int64_t send_id) {
    std::vector<c10::intrusive_ptr<c10d::Work>> works;
    {
        std::lock_guard<std::mutex> lk(g_sends_m);
        auto it = g_sends.find(send_id);
        if (it == g_sends.end()) return;  // failed job (its error is raised by rw_check)
        works = std::move(it->second);
        g_sends.erase(it);
    }
    pybind11::gil_scoped_release no_gil;
    for (auto& w : works) w->wait();
}

// Python-level gloo call in program order: host_begin blocks (GIL released) until every earlier job has run and the
// worker waits for host_end.
int64_t rw_host_begin() {
    Worker& w = worker();
    int64_t ticket;
    {
        std::lock_guard<std::mutex> lk(w.m);
        ticket = w.host_next++;
    }
    w.push([&w, ticket]() {
        std::unique_lock<std::mutex> lk(w.m);
        w.host_turn = ticket;
        w.host_running = true;
        w.cv.notify_all();
        w.cv.wait(lk, [&w] { return !w.host_running; });
    });
    pybind11::gil_scoped_release no_gil;
    std::unique_lock<std::mutex> lk(w.m);
    w.cv.wait(lk, [&w, ticket] { return w.host_turn == ticket && w.host_running; });
    return ticket;
}
void rw_host_end(int64_t ticket) {
    Worker& w = worker();
    {
        std::lock_guard<std::mutex> lk(w.m);
        TORCH_CHECK(w.host_turn == ticket && w.host_running, "rehearsal worker: host_end out of turn");
        w.host_running = false;
    }
    w.cv.notify_all();
}
// Raises the first error a job hit (collectives after it already opened their gates with unwritten results).
void rw_check() {
    Worker& w = worker();
    std::lock_guard<std::mutex> lk(w.m);
    TORCH_CHECK(w.error.empty(), "asynchronous rehearsal collective failed: ", w.error);
}
// Waits (GIL released) until every job queued so far has run.
void rw_drain() {
    const int64_t t = rw_host_begin();
    rw_host_end(t);
}

void register_rehearsal(pybind11::module& m) {
    m.def("rw_collective", &rw_collective, "rehearsal worker: queue one gloo collective behind a stream gate",
          pybind11::call_guard<pybind11::gil_scoped_release>());
    m.def("rw_host_begin", &rw_host_begin, "rehearsal worker: wait for this Python-level gloo call's turn");
    m.def("rw_host_end", &rw_host_end, "rehearsal worker: a Python-level gloo call is done");
    m.def("rw_check", &rw_check, "rehearsal worker: raise the first failed job's error");
    m.def("rw_drain", &rw_drain, "rehearsal worker: wait for every queued job");
    m.def("rw_p2p_send", &rw_p2p_send, "rehearsal worker: queue posting pipeline sends behind an event",
          pybind11::call_guard<pybind11::gil_scoped_release>());
    m.def("rw_p2p_recv", &rw_p2p_recv, "rehearsal worker: queue pipeline receives behind a stream gate",
          pybind11::call_guard<pybind11::gil_scoped_release>());
    m.def("rw_send_wait", &rw_send_wait, "rehearsal worker: wait for a send batch (inside a host turn)");
}
