// rconn_bench — throughput of the RConn-shaped adapter (include/rsk_rconn.h) from C++: n payloads of
// P bytes through rsk_rconn_output (frames land in the send callback), then those frames through
// rsk_rconn_onrecv (VALID payloads land in the recv callback).  Per-call host work (payload copy,
// staging, callbacks) is included; one JSON line.
//   tools/rconn_bench [n=1048576] [payload=1400] [batch=65536]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

int main(int argc, char **argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1048576;
    const int P = argc > 2 ? atoi(argv[2]) : 1400;
    const uint32_t batch = argc > 3 ? (uint32_t)atoi(argv[3]) : 65536;
    const char key[] = "hello135";
    rsk_rconn *r = rsk_rconn_create(reinterpret_cast<const uint8_t *>(key), 8, 0, batch);
    if (!r) {
        fprintf(stderr, "rsk_rconn_create failed: %s\n", rsk_last_error());
        return 1;
    }
    Sink sink;
    sink.pitch = 1504;
    sink.frames.assign(n * sink.pitch, 0);
    sink.flen.assign(n, 0);
    rsk_rconn_set_callbacks(r, on_send, on_reset, on_recv, &sink);
    std::vector<uint8_t> pay((size_t)P * 64);
    for (size_t k = 0; k < pay.size(); ++k) pay[k] = (uint8_t)(k * 131 + 7);
    const uint8_t id[8] = {'a', 'b', 'c', 'd', 'e', 'f', 'g', 'h'};
    auto now = [] { return std::chrono::steady_clock::now(); };
    // warm-up batch
    for (size_t i = 0; i < batch && i < n; ++i)
        rsk_rconn_output(r, P, reinterpret_cast<const char *>(pay.data() + (i % 64) * P), 0, id, 1, 0x10002711, (void *)i);
    rsk_rconn_flush(r);
    sink.sent = 0;
    auto t0 = now();
    for (size_t i = 0; i < n; ++i)
        if (rsk_rconn_output(r, P, reinterpret_cast<const char *>(pay.data() + (i % 64) * P), 0, id, (uint32_t)i,
                             0x10002711, (void *)i) != 31 + P)
            return 2;
    if (rsk_rconn_flush(r)) return 3;
    const double t_out = std::chrono::duration<double>(now() - t0).count();
    if (sink.sent != n) return 4;
    t0 = now();
    for (size_t i = 0; i < n; ++i)
        rsk_rconn_onrecv(r, sink.flen[i], reinterpret_cast<const char *>(sink.frames.data() + i * sink.pitch), 0,
                         (void *)i);
    if (rsk_rconn_flush(r)) return 5;
    const double t_in = std::chrono::duration<double>(now() - t0).count();
    if (sink.recv_valid != n || sink.recv_bytes != (uint64_t)n * P) return 6;
    printf("{\"adapter\": \"rsk_rconn\", \"packets\": %zu, \"payload\": %d, \"batch\": %u, "
           "\"output_Mpkt_s\": %.1f, \"onrecv_Mpkt_s\": %.1f, \"threads\": 1}\n",
           n, P, batch, n / t_out / 1e6, n / t_in / 1e6);
    rsk_rconn_destroy(r);
    return 0;
}
