/*
 * ref_parse_harness.cpp — TEST INFRASTRUCTURE ONLY.
 *
 * Runs the REFERENCE's own receive parse, RawTcp::RawInput (conn/RawTcp.cpp:138-237), compiled
 * from /root/reference by oracle/Makefile (`make -C oracle ref` -> oracle/_ref/
 * librsk_ref_parse.so; nothing from the reference is copied here).  As SURVEY.md §8c describes,
 * a subclass overrides the virtual cap2uv (RawTcp.h:51) to capture what RawInput hands over, and
 * the object is built with the 4-argument constructor and never Init()ed / Close()d.
 *
 * The library links the reference objects RawInput needs (RawTcp, IConn, TcpAckPool, TcpInfo,
 * ConnInfo, rsutil, enc, ...) against the vendored HEADERS only.  The libnet / pcap / service
 * functions that RawInput never calls (libnet_init, libnet_build_*, CapUtil::DataLink,
 * RouteService::..., SyncConnFactory::...) stay unresolved: the library is loaded with lazy
 * binding (RTLD_LAZY), so they are never bound; no stand-in is written for any of them.
 *
 * Private members (RawTcp::mDatalink, TcpAckPool::mInfoPool) are reached by compiling the two
 * class headers with `private` spelled `public` in THIS translation unit only (layout unchanged).
 */
#include <cstdint>
#include <cstring>
#include <condition_variable>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include <libnet.h>
#include <pcap.h>
#include <uv.h>
#include <plog/Log.h>
#include <plog/Appenders/IAppender.h>

#include "rscomm.h"
#include "rcommon.h"
#include "conn/IConn.h"
#include "src/service/IRouteObserver.h"
#include "src/service/ITimerObserver.h"
#include "bean/TcpInfo.h"
#include "src/util/TcpCmpFn.h"

#define private public
#include "conn/RawTcp.h"
#include "net/TcpAckPool.h"
#undef private

namespace {

struct Capture {
    int called = 0;
    TcpInfo info;
    long pay_off = 0;
    int payload_len = 0;
    int base_ret = 0;  // RawTcp::cap2uv's own return (size check), 99 = not run (negative length)
};

class ProbeTcp : public RawTcp {
public:
    ProbeTcp(TcpAckPool *pool, bool server) : RawTcp("lo", nullptr, pool, server) {}
    const uint8_t *pkt = nullptr;
    Capture cap;

protected:
    int cap2uv(const TcpInfo *info, const char *payload, int payload_len) override {
        cap.called = 1;
        cap.info = *info;
        cap.pay_off = (long)((const uint8_t *)payload - pkt);
        cap.payload_len = payload_len;
        // The base cap2uv: size check (RawTcp.cpp:240, in size_t), Encode into a 1500-B buffer,
        // memcpy, then mSyncConn == nullptr -> -1.  A payload_len in [-32, 0) passes the size_t check
        // and reaches memcpy with a negative length (undefined), so it is not run for those (99).
        const bool ub = payload_len < 0 && payload_len >= -(int)(2 * sizeof(SA4));
        cap.base_ret = ub ? 99 : RawTcp::cap2uv(info, payload, payload_len);
        return 0;
    }
};

bool g_plog = false;

}  // namespace

extern "C" {

/* One captured packet through RawTcp::RawInput.  out[] (uint32):
 *  0 ret   1 cap2uv called   2..8 info src,dst,sp,dp,seq,ack,flag   9 payload offset in pkt
 * 10 payload_len (int)  11 base cap2uv ret (int)  12 ack-pool entries  13..19 entry src..flag */
int ref_rawinput(const uint8_t *pkt, uint32_t wire_len, uint32_t cap_len, int datalink, int is_server,
                 int with_ack_pool, uint32_t *out) {
    if (!g_plog) {  // RawTcp.cpp:197 calls plog::get(); severity none logs nothing
        plog::init(plog::none);
        g_plog = true;
    }
    TcpAckPool pool(1000);
    ProbeTcp t(with_ack_pool ? &pool : nullptr, is_server != 0);
    t.mDatalink = datalink == 0 ? DLT_NULL : DLT_EN10MB;
    t.pkt = pkt;
    pcap_pkthdr hdr;
    std::memset(&hdr, 0, sizeof hdr);
    hdr.len = wire_len;
    hdr.caplen = cap_len;
    std::memset(out, 0, 20 * sizeof(uint32_t));
    out[0] = (uint32_t)t.RawInput(nullptr, &hdr, pkt);
    const Capture &c = t.cap;
    out[1] = (uint32_t)c.called;
    if (c.called) {
        out[2] = c.info.src; out[3] = c.info.dst; out[4] = c.info.sp; out[5] = c.info.dp;
        out[6] = c.info.seq; out[7] = c.info.ack; out[8] = c.info.flag;
        out[9] = (uint32_t)c.pay_off;
        out[10] = (uint32_t)c.payload_len;
        out[11] = (uint32_t)c.base_ret;
    }
    out[12] = (uint32_t)pool.mInfoPool.size();
    if (!pool.mInfoPool.empty()) {
        const TcpInfo &e = pool.mInfoPool.begin()->first;
        out[13] = e.src; out[14] = e.dst; out[15] = e.sp; out[16] = e.dp;
        out[17] = e.seq; out[18] = e.ack; out[19] = e.flag;
    }
    return 0;
}

}  // extern "C"
