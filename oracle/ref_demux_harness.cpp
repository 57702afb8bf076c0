/*
 * ref_demux_harness.cpp — TEST INFRASTRUCTURE ONLY.
 *
 * Runs the REFERENCE's own receive routing over a batch of decoded packets, compiled from
 * /root/reference by oracle/Makefile (`make -C oracle ref` -> oracle/_ref/librsk_ref_demux.so;
 * nothing from the reference is copied here):
 *   server: ServerGroup::OnRecv   by IdBuf            (server/ServerGroup.cpp:44-63)
 *        -> IAppGroup::Input      by cmd              (conn/IAppGroup.cpp:76-96)
 *        -> INetGroup::Input      by connKey          (conn/INetGroup.cpp:57-83)
 *        -> INetConn::OnRecv -> IConn::OnRecv -> SubGroup::OnRecv by BuildConvKey(dst, conv)
 *                                                      (server/SubGroup.cpp:31-51)
 *   client: IAppGroup::Input      by cmd
 *        -> INetGroup::Input      by connKey (pre-existing conns only: CNetGroup::CreateNetConn
 *                                  returns nullptr, client/CNetGroup.cpp)
 *        -> ClientGroup::OnRecv   by conv             (client/ClientGroup.cpp:65-80)
 *
 * Recording stand-ins sit only at the ends of those chains, behind the reference's own virtual
 * interfaces:
 *   - INetGroup::CreateNetConn (pure virtual, INetGroup.h:35) returns a recording INetConn;
 *   - the leaf conns (SConn in the reference) are recording IConns whose OnRecv records and returns
 *     nread; the client's leaves are real CConn objects (conn/CConn.cpp) with OnRecv recording;
 *   - IReset / INetConnKeepAlive (pure interfaces, callbacks/IReset.h, INetConnKeepAlive.h) are
 *     recording implementations; IAppGroup::SendConvRst (virtual) is recorded on the client;
 *   - ServerGroup::newConn / SubGroup::newConn construct SNetGroup + SubGroup / SConn and Init() them,
 *     which needs a libuv loop, the net manager and ConfManager: the harness overrides the virtual
 *     IGroup::ConnOfKey (IGroup.h) to construct on the FIRST MISS instead, so the lookup key, the
 *     lookup order and the dispatch around it are the reference's own code.
 *   - Init() of the groups is replaced by the parts of it that wire the chain (IGroup::Init, and
 *     IAppGroup::Init's two callback bindings, IAppGroup.cpp:38-41) — the rest registers services.
 * Private members (IAppGroup::mResetHelper / mKeepAlive, INetGroup::mDefaultFakeConn,
 * ClientGroup::mConvMap) are reached by compiling the class headers with `private` (and
 * `protected`: IGroup::mConns) spelled `public` in THIS translation unit only (layout unchanged), as ref_parse_harness.cpp does.
 * Functions none of this calls (uv, libnet, services) stay unresolved; RTLD_LAZY.
 */
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <sys/un.h>

#include <array>
#include <cassert>
#include <cstdint>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include <uv.h>
#include <plog/Log.h>

#include "rscomm.h"
#include "rcommon.h"
#include "bean/EncHead.h"
#include "bean/ConnInfo.h"
#include "bean/TcpInfo.h"
#include "callbacks/IReset.h"
#include "callbacks/INetConnKeepAlive.h"
#include "conn/IConn.h"
#include "conn/INetConn.h"
#include "conn/CConn.h"
#include "util/rsutil.h"

#define private public
#define protected public
#include "conn/IGroup.h"
#include "conn/INetGroup.h"
#include "conn/IAppGroup.h"
#include "server/ServerGroup.h"
#include "server/SubGroup.h"
#include "client/ClientGroup.h"
#undef protected
#undef private

using namespace std::placeholders;

namespace {

/* ---- event log ---------------------------------------------------------------------------- */
enum EvKind : int64_t {
    EV_CREATE = 1,      /* conn created               (conn, pkt)                               */
    EV_DELIVER = 2,     /* conn's OnRecv ran          (conn, pkt)                               */
    EV_RST_IN = 3,      /* IReset::Input(cmd)         (-1,   pkt, cmd)                          */
    EV_KA_IN = 4,       /* INetConnKeepAlive::Input   (-1,   pkt, cmd)                          */
    EV_CONV_RST = 5,    /* IAppGroup::SendConvRst     (-1,   pkt, conv)                         */
    EV_NETCONN_RST = 6, /* IReset::SendNetConnRst     (-1,   pkt, connKey)                      */
    EV_DEFAULT_IN = 7,  /* INetGroup's default conn   (-1,   pkt)                               */
};
enum Level : int { LV_GROUP = 0, LV_NET = 1, LV_LEAF = 2 };

struct Conn {
    int level;
    int parent;       /* conn id of the owning group (server), -1 at the top */
    std::string key;  /* IConn::Key() */
};

struct Log {
    std::vector<int64_t> ev;  /* 4 per event: kind, conn, pkt, aux */
    std::vector<Conn> conns;
    int64_t pkt = -1;
    void add(int64_t kind, int64_t conn, int64_t aux = 0) {
        ev.push_back(kind); ev.push_back(conn); ev.push_back(pkt); ev.push_back(aux);
    }
    int new_conn(int level, int parent, const std::string &key) {
        conns.push_back(Conn{level, parent, key});
        int id = (int)conns.size() - 1;
        add(EV_CREATE, id);
        return id;
    }
};
Log *g_log = nullptr;

/* ---- recording ends of the chains ---------------------------------------------------------- */
class RecLeaf : public IConn {  /* the server's SConn position */
public:
    RecLeaf(const std::string &key, int id) : IConn(key), mId(id) {}
    int OnRecv(ssize_t nread, const rbuf_t &rbuf) override {
        g_log->add(EV_DELIVER, mId);
        return (int)nread;
    }
    int mId;
};

class RecCConn : public CConn {  /* the client's real CConn, OnRecv recorded */
public:
    RecCConn(const std::string &key, const SA *addr, uint32_t conv, int id) : CConn(key, addr, conv), mId(id) {}
    int OnRecv(ssize_t nread, const rbuf_t &rbuf) override {
        g_log->add(EV_DELIVER, mId);
        return (int)nread;
    }
    int mId;
};

class RecNetConn : public INetConn {  /* FakeTcp / FakeUdp position */
public:
    RecNetConn(IntKeyType key, const ConnInfo &info, int id) : INetConn(key), mInfo(info), mId(id) {
        mInfo.head = nullptr;
    }
    bool IsUdp() override { return mInfo.IsUdp(); }
    ConnInfo *GetInfo() override { return &mInfo; }
    int OnRecv(ssize_t nread, const rbuf_t &rbuf) override {  /* as FakeTcp::OnRecv: forward up */
        g_log->add(EV_DELIVER, mId);
        return INetConn::OnRecv(nread, rbuf);
    }
    TcpInfo mInfo;
    int mId;
};

class RecDefault : public IConn {  /* INetGroup::mDefaultFakeConn */
public:
    RecDefault() : IConn("default") {}
    int OnRecv(ssize_t nread, const rbuf_t &rbuf) override {
        g_log->add(EV_DEFAULT_IN, -1);
        return 0;
    }
};

class RecReset : public IReset {
public:
    void Close() override {}
    int Input(uint8_t cmd, ssize_t nread, const rbuf_t &rbuf) override {
        g_log->add(EV_RST_IN, -1, cmd);
        return (int)nread;
    }
    int SendConvRst(uint32_t conv) override { g_log->add(EV_CONV_RST, -1, conv); return 0; }
    int SendNetConnRst(const ConnInfo &src, IntKeyType key) override {
        g_log->add(EV_NETCONN_RST, -1, (int64_t)key);
        return 0;
    }
    int OnRecvNetConnRst(const ConnInfo &src, IntKeyType key) override { return 0; }
    int OnRecvConvRst(const ConnInfo &src, uint32_t rstConv) override { return 0; }
};

class RecKeepAlive : public INetConnKeepAlive {
public:
    int Init() override { return 0; }
    int Input(uint8_t cmd, ssize_t nread, const rbuf_t &rbuf) override {
        g_log->add(EV_KA_IN, -1, cmd);
        return (int)nread;
    }
    int SendResponse(IntKeyType connKey) override { return 0; }
    int SendRequest(IntKeyType connKey) override { return 0; }
    int Close() override { return 0; }
    int OnRecvResponse(IntKeyType connKey) override { return 0; }
    int RemoveRequest(IntKeyType connkey) override { return 0; }
    int RemoveAllRequest() override { return 0; }
};

/* INetGroup with the pure-virtual CreateNetConn: the server creates on demand (SNetGroup, UDP and
 * TCP with a pooled tcp), the client never does (CNetGroup). */
class RecNetGroup : public INetGroup {
public:
    RecNetGroup(const std::string &groupId, bool on_demand, int owner)
        : INetGroup(groupId, nullptr), mOnDemand(on_demand), mOwner(owner) {}
    INetConn *CreateNetConn(IntKeyType key, const ConnInfo *info) override {
        if (!mOnDemand) return nullptr;
        int id = g_log->new_conn(LV_NET, mOwner, std::to_string(key));
        auto *c = new RecNetConn(key, *info, id);
        c->Init();
        return c;
    }
    bool mOnDemand;
    int mOwner;
};

/* The chain wiring of INetGroup::Init / IAppGroup::Init (IAppGroup.cpp:27-48) without the
 * services: handler, ConfManager, keep-alive timers. */
void wire_app(IAppGroup *app, RecNetGroup *net) {
    app->IGroup::Init();
    net->IGroup::Init();
    net->mDefaultFakeConn = new RecDefault();
    net->mDefaultFakeConn->Init();
    net->SetOutputCb(std::bind(&IConn::Output, app, _1, _2));
    net->SetOnRecvCb(std::bind(&IConn::OnRecv, app, _1, _2));
    app->mResetHelper = new RecReset();
    app->mKeepAlive = new RecKeepAlive();
}

void unwire_app(IAppGroup *app, RecNetGroup *net) {
    std::vector<IConn *> nets;
    for (auto &e : net->mConns) nets.push_back(e.second);
    for (IConn *c : nets) { net->RemoveConn(c); c->Close(); delete c; }
    net->mDefaultFakeConn->Close();
    delete net->mDefaultFakeConn;
    net->mDefaultFakeConn = nullptr;
    net->IConn::Close();
    delete app->mResetHelper; app->mResetHelper = nullptr;
    delete app->mKeepAlive; app->mKeepAlive = nullptr;
    std::vector<IConn *> leaves;
    for (auto &e : app->mConns) leaves.push_back(e.second);
    for (IConn *c : leaves) { app->IGroup::RemoveConn(c); c->Close(); delete c; }
    app->IConn::Close();
}

/* SubGroup whose leaf construction (SubGroup::newConn -> SConn) happens on the first miss. */
class HSubGroup : public SubGroup {
public:
    HSubGroup(const std::string &groupId, const struct sockaddr *target, RecNetGroup *net, int id)
        : SubGroup(groupId, nullptr, target, net, nullptr), mId(id) {}
    IConn *ConnOfKey(const std::string &key) override {
        IConn *c = IGroup::ConnOfKey(key);
        if (c) return c;
        int id = g_log->new_conn(LV_LEAF, mId, key);
        auto *leaf = new RecLeaf(key, id);
        leaf->Init();
        AddConn(leaf, nullptr, nullptr);
        return leaf;
    }
    int Input(ssize_t nread, const rbuf_t &rbuf) override {  /* the group's own delivery */
        g_log->add(EV_DELIVER, mId);
        return IAppGroup::Input(nread, rbuf);
    }
    int mId;
};

/* ServerGroup whose SubGroup construction (ServerGroup::newConn) happens on the first miss. */
class HServerGroup : public ServerGroup {
public:
    explicit HServerGroup(const struct sockaddr *target) : ServerGroup("server01", nullptr, target, nullptr, nullptr) {}
    IConn *ConnOfKey(const std::string &key) override {
        IConn *c = IGroup::ConnOfKey(key);
        if (c) return c;
        int id = g_log->new_conn(LV_GROUP, -1, key);
        auto *net = new RecNetGroup(key, true, id);
        auto *sub = new HSubGroup(key, mTarget, net, id);
        wire_app(sub, net);
        AddConn(sub, nullptr, nullptr);  /* ServerGroup.cpp:76-77 binds its Send as the output */
        mSubs.push_back(sub);
        mNets.push_back(net);
        return sub;
    }
    ~HServerGroup() {
        for (size_t i = 0; i < mSubs.size(); i++) {
            IGroup::RemoveConn(mSubs[i]);
            unwire_app(mSubs[i], mNets[i]);
            mSubs[i]->mFakeNetGroup = nullptr;
            delete mNets[i];
            delete mSubs[i];
        }
        IConn::Close();
        if (mTarget) { free(mTarget); mTarget = nullptr; }
    }
    std::vector<HSubGroup *> mSubs;
    std::vector<RecNetGroup *> mNets;
};

class HClientGroup : public ClientGroup {
public:
    explicit HClientGroup(RecNetGroup *net) : ClientGroup("client01", "", "", 0, nullptr, net, nullptr) {}
    int SendConvRst(uint32_t conv) override {  /* ClientGroup.cpp:76 for an unknown conv */
        g_log->add(EV_CONV_RST, -1, conv);
        return 0;
    }
};

bool g_plog = false;

}  // namespace

extern "C" {

/* Route the VALID packets of a decoded batch through the reference's groups, in the order given.
 *   stack 0 = server (ServerGroup -> SubGroup/IAppGroup -> INetGroup -> SubGroup::OnRecv),
 *   stack 1 = client (ClientGroup/IAppGroup -> INetGroup -> ClientGroup::OnRecv); the client's
 *   net conns (known_keys) and CConns (known_convs) exist before the batch, as after connecting.
 * order[0..n_order) lists packet indices; a packet with valid[i] == 0 (RConn::OnRecv did not pass
 * it up: DROP or CLOSE_NOTIFY) is skipped.
 * Outputs: ret[i] = the top-level call's return for each routed packet (untouched otherwise);
 * ev[4*k ..] = (kind, conn, pkt, aux) for k < *n_ev; conns: conn_level[c], conn_parent[c] and
 * conn_key[c*48 ..] (IConn::Key(), zero padded, conn_key_len[c]) for c < *n_conn.
 * Returns 0, or -1 when a capacity is exceeded. */
int ref_demux_run(int stack, uint32_t n, const int8_t *valid, const uint8_t *cmd, const uint8_t *id,
                  const uint32_t *conv, const uint64_t *conn_key, const uint32_t *dst,
                  const uint32_t *order, uint32_t n_order, const uint64_t *known_keys, uint32_t n_known_keys,
                  const uint32_t *known_convs, uint32_t n_known_convs, int32_t *ret, int64_t *ev,
                  uint32_t ev_cap, uint32_t *n_ev, int32_t *conn_level, int32_t *conn_parent, uint8_t *conn_key_out,
                  uint32_t *conn_key_len, uint32_t conn_cap, uint32_t *n_conn) {
    if (!g_plog) {  /* the groups log through plog; severity none logs nothing */
        plog::init(plog::none);
        g_plog = true;
    }
    Log log;
    g_log = &log;
    struct sockaddr_in target;
    std::memset(&target, 0, sizeof target);
    target.sin_family = AF_INET;
    target.sin_port = htons(10001);
    target.sin_addr.s_addr = htonl(0x7f000001);

    std::unique_ptr<HServerGroup> srv;
    std::unique_ptr<HClientGroup> cli;
    RecNetGroup *cnet = nullptr;
    IConn *top = nullptr;
    if (stack == 0) {
        srv.reset(new HServerGroup((const struct sockaddr *)&target));
        srv->IGroup::Init();  /* ServerGroup::Init also registers a NetService observer */
        top = srv.get();
    } else {
        cnet = new RecNetGroup("client", false, -1);
        cli.reset(new HClientGroup(cnet));
        wire_app(cli.get(), cnet);
        TcpInfo info;
        for (uint32_t k = 0; k < n_known_keys; k++) {  /* connected fake-tcp conns */
            int cid = log.new_conn(LV_NET, -1, std::to_string(known_keys[k]));
            auto *c = new RecNetConn(known_keys[k], info, cid);
            c->Init();
            cnet->AddNetConn(c);
        }
        for (uint32_t k = 0; k < n_known_convs; k++) {  /* ClientGroup::newConn (ClientGroup.cpp:206-217) */
            struct sockaddr_in a = target;
            a.sin_port = htons((uint16_t)(20000 + k));
            std::string key = CConn::BuildKey((const SA *)&a);
            int cid = log.new_conn(LV_LEAF, -1, key);
            auto *c = new RecCConn(key, (const SA *)&a, known_convs[k], cid);
            c->Init();
            cli->AddConn(c, nullptr, nullptr);
            cli->mConvMap.insert({known_convs[k], c});
        }
        top = cli.get();
    }
    /* setup events are not part of the batch */
    log.ev.clear();

    char payload[64];
    std::memset(payload, 0x5a, sizeof payload);
    for (uint32_t j = 0; j < n_order; j++) {
        const uint32_t i = order[j];
        if (i >= n || !valid[i]) continue;
        EncHead head;
        head.SetCmd(cmd[i]);
        IdBufType idb;
        std::memcpy(idb.data(), id + 8ull * i, 8);
        head.SetIdBuf(idb);
        head.SetConv(conv[i]);
        head.SetConnKey(conn_key[i]);
        TcpInfo info;  /* RConn::OnRecv hands the decoded head up with the packet's TcpInfo */
        info.src = 0x0100000a;
        info.dst = dst[i];
        info.sp = 10001;
        info.dp = 43932;
        info.head = &head;
        const rbuf_t rb = new_buf(32, payload, &info);
        log.pkt = i;
        /* RConn's recv callback is bound to IConn::Input of the group above it (IGroup.cpp:36) */
        ret[i] = top->Input(32, rb);
    }

    if (stack == 1) {
        for (auto &e : cli->mConvMap) { cli->IGroup::RemoveConn(e.second); e.second->Close(); delete e.second; }
        cli->mConvMap.clear();
        unwire_app(cli.get(), cnet);
        cli->mFakeNetGroup = nullptr;
        delete cnet;
        cli.reset();
    } else {
        srv.reset();
    }
    g_log = nullptr;

    if (log.ev.size() / 4 > ev_cap || log.conns.size() > conn_cap) return -1;
    std::memcpy(ev, log.ev.data(), log.ev.size() * sizeof(int64_t));
    *n_ev = (uint32_t)(log.ev.size() / 4);
    for (size_t c = 0; c < log.conns.size(); c++) {
        conn_level[c] = log.conns[c].level;
        conn_parent[c] = log.conns[c].parent;
        const std::string &k = log.conns[c].key;
        const size_t m = k.size() < 48 ? k.size() : 48;
        std::memset(conn_key_out + 48 * c, 0, 48);
        std::memcpy(conn_key_out + 48 * c, k.data(), m);
        conn_key_len[c] = (uint32_t)m;
    }
    *n_conn = (uint32_t)log.conns.size();
    return 0;
}

}  // extern "C"
