// rconn_bench — throughput of the RConn-shaped adapter (include/rsk_rconn.h) from C++: n payloads of
// P bytes through rsk_rconn_output (frames land in the send callback), then those frames through
// rsk_rconn_onrecv (VALID payloads land in the recv callback).  Per-call host work (payload copy,
// staging, callbacks) is included; one JSON line.  With threads = T > 1, T calling threads each drive
// their own adapter (own context and stream, as one rsk_rconn per capture / loop thread would) over
// n / T packets; the rates are n over the slowest thread's time, all threads released together.
//   tools/rconn_bench [n=1048576] [payload=1400] [batch=65536] [threads=1]
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../include/rsk_rconn.h"

struct Sink {
    std::vector<uint8_t> frames;
    std::vector<int> flen;
    size_t pitch = 0;
    uint64_t sent = 0, recv_valid = 0, recv_bytes = 0;
    bool keep = true;
};

static int on_send(const char *f, int len, void *user, void *arg) {
    Sink *s = static_cast<Sink *>(arg);
    const size_t i = (size_t)(uintptr_t)user;
    if (s->keep) {
        std::memcpy(s->frames.data() + i * s->pitch, f, (size_t)len);
        s->flen[i] = len;
    }
    ++s->sent;
    return 0;
}
static int on_reset(void *, void *) { return 0; }
static int on_recv(int status, uint8_t, uint8_t, const uint8_t *, uint32_t, uint64_t, const char *, int plen, void *,
                   void *arg) {
    Sink *s = static_cast<Sink *>(arg);
    if (status == RSK_RECV_VALID) {
        ++s->recv_valid;
        s->recv_bytes += (uint64_t)plen;
    }
    return 0;
}

struct Run {
    size_t n = 0;
    int P = 0;
    uint32_t batch = 0;
    rsk_rconn *r = nullptr;
    Sink sink;
    double t_out = 0, t_in = 0;
    int rc = 0;
};

using Clock = std::chrono::steady_clock;

// Output then OnRecv of run.n packets; `go` releases the timed Output loop, `mid` the OnRecv loop, so
// that every thread's two phases start together.
static void drive(Run &run, std::atomic<int> &go, std::atomic<int> &mid, int threads) {
    const size_t n = run.n;
    const int P = run.P;
    rsk_rconn *r = run.r;
    Sink &sink = run.sink;
    std::vector<uint8_t> pay((size_t)P * 64);
    for (size_t k = 0; k < pay.size(); ++k) pay[k] = (uint8_t)(k * 131 + 7);
    const uint8_t id[8] = {'a', 'b', 'c', 'd', 'e', 'f', 'g', 'h'};
    // warm-up batch
    for (size_t i = 0; i < run.batch && i < n; ++i)
        rsk_rconn_output(r, P, reinterpret_cast<const char *>(pay.data() + (i % 64) * P), 0, id, 1, 0x10002711, (void *)i);
    rsk_rconn_flush(r);
    sink.sent = 0;
    go.fetch_add(1);
    while (go.load() < threads) std::this_thread::yield();
    auto t0 = Clock::now();
    for (size_t i = 0; i < n; ++i)
        if (rsk_rconn_output(r, P, reinterpret_cast<const char *>(pay.data() + (i % 64) * P), 0, id, (uint32_t)i,
                             0x10002711, (void *)i) != 31 + P) {
            run.rc = 2;
            break;
        }
    if (!run.rc && rsk_rconn_flush(r)) run.rc = 3;
    run.t_out = std::chrono::duration<double>(Clock::now() - t0).count();
    if (!run.rc && sink.sent != n) run.rc = 4;
    mid.fetch_add(1);
    while (mid.load() < threads) std::this_thread::yield();
    if (run.rc) return;
    t0 = Clock::now();
    for (size_t i = 0; i < n; ++i)
        rsk_rconn_onrecv(r, sink.flen[i], reinterpret_cast<const char *>(sink.frames.data() + i * sink.pitch), 0,
                         (void *)i);
    if (rsk_rconn_flush(r)) run.rc = 5;
    run.t_in = std::chrono::duration<double>(Clock::now() - t0).count();
    if (!run.rc && (sink.recv_valid != n || sink.recv_bytes != (uint64_t)n * P)) run.rc = 6;
}

int main(int argc, char **argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1048576;
    const int P = argc > 2 ? atoi(argv[2]) : 1400;
    const uint32_t batch = argc > 3 ? (uint32_t)atoi(argv[3]) : 65536;
    const int threads = argc > 4 ? std::max(1, atoi(argv[4])) : 1;
    const char key[] = "hello135";
    std::vector<Run> runs(threads);
    for (int t = 0; t < threads; ++t) {
        Run &run = runs[t];
        run.n = n * (t + 1) / threads - n * t / threads;
        run.P = P;
        run.batch = batch;
        run.r = rsk_rconn_create(reinterpret_cast<const uint8_t *>(key), 8, 0, batch);
        if (!run.r) {
            fprintf(stderr, "rsk_rconn_create failed: %s\n", rsk_last_error());
            return 1;
        }
        run.sink.pitch = 1504;
        run.sink.frames.assign(run.n * run.sink.pitch, 0);
        run.sink.flen.assign(run.n, 0);
        rsk_rconn_set_callbacks(run.r, on_send, on_reset, on_recv, &run.sink);
    }
    std::atomic<int> go{0}, mid{0};
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) th.emplace_back(drive, std::ref(runs[t]), std::ref(go), std::ref(mid), threads);
    for (auto &x : th) x.join();
    double t_out = 0, t_in = 0;
    for (auto &run : runs) {
        if (run.rc) return run.rc;
        t_out = std::max(t_out, run.t_out);
        t_in = std::max(t_in, run.t_in);
        rsk_rconn_destroy(run.r);
    }
    printf("{\"adapter\": \"rsk_rconn\", \"packets\": %zu, \"payload\": %d, \"batch\": %u, "
           "\"output_Mpkt_s\": %.1f, \"onrecv_Mpkt_s\": %.1f, \"threads\": %d}\n",
           n, P, batch, n / t_out / 1e6, n / t_in / 1e6, threads);
    return 0;
}
