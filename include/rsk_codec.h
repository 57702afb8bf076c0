/*
 * rsk_codec.h — C ABI of the MI355X framing codec (drop-in for rsock's per-packet codec path).
 *
 * Every entry point is extern "C", takes plain pointers and sizes, and returns 0 or a negative
 * error code.  Batch entry points are stream-ordered (the `stream` argument is a hipStream_t,
 * passed as void* so this header needs no HIP include; NULL = the legacy default stream) and take
 * no ownership: the caller owns every device and host buffer.  All batch array pointers are
 * DEVICE pointers unless a comment says otherwise.  An empty batch (n == 0) is a no-op that may
 * pass null arrays (the ctx and the in/out structs must still be given); it zeroes a given
 * n_valid / n_match / n_seg count.
 *
 * Reference interfaces replaced (paths relative to the rsock tree):
 *   rsk_compute_hash      <- char* compute_hash(char*, const std::string&, const char*, int)   util/rhash.h:17, util/rhash.cpp:20-41
 *   rsk_hash_equal        <- bool hash_equal(const char*, const std::string&, const char*, int) util/rhash.h:13, util/rhash.cpp:71-92
 *   rsk_enchead_enc2buf   <- char* EncHead::Enc2Buf(char*, int)                               bean/EncHead.h:40, bean/EncHead.cpp:9-24
 *   rsk_enchead_decodebuf <- static const char* EncHead::DecodeBuf(EncHead&, const char*, int) bean/EncHead.h:38, bean/EncHead.cpp:39-55
 *   rsk_encode_batch      <- int RConn::Output(ssize_t, const rbuf_t&), framing part          conn/RConn.h:37, conn/RConn.cpp:87-105
 *   rsk_decode_batch      <- int RConn::OnRecv(ssize_t, const rbuf_t&)                        conn/RConn.h:34, conn/RConn.cpp:64-85
 *   rsk_parse_decode_batch<- int RawTcp::RawInput(u_char*, const pcap_pkthdr*, const u_char*) conn/RawTcp.h:38, conn/RawTcp.cpp:138-237
 *   rsk_parse_decode_slots_batch <- the same on host-staged header slots (payloads stay in the capture buffer)
 *                            + RawTcp::cap2uv size check (RawTcp.cpp:239-244) fused with RConn::OnRecv
 *   rsk_tcpinfo_encode_batch <- char* TcpInfo::Encode(char*, int) (21-B hand-off record)      bean/TcpInfo.cpp:20-32, bean/ConnInfo.cpp:12-20
 *   rsk_syncinput_decode_batch <- RawTcp::syncInput -> TcpInfo::Decode -> RConn::OnRecv     conn/RawTcp.cpp:262-276, bean/TcpInfo.cpp:35-47
 *   rsk_encode_wire_batch <- RConn::Output + RawTcp::SendRawTcp -> libnet_build_tcp/ipv4     conn/RawTcp.cpp:280-341
 *   rsk_key_for_tcp/udp   <- KeyGenerator::KeyForTcp / KeyForUdp                              src/util/KeyGenerator.cpp:16-36
 *   rsk_capture_filter_batch <- the pcap filter RCap installs: BuildFilterStr("tcp", srcIp, dstIp, srcPorts,
 *                            dstPorts, isServer) (cap/cap_util.cpp:67-144, cap/RCap.cpp:64-88) evaluated
 *                            per captured packet; rsk_filter_str renders the same string
 *   rsk_filter_parse_decode_batch <- that filter fused with RawTcp::RawInput + RConn::OnRecv (one pass)
 *   rsk_tcp_send_seq_batch <- FakeTcp::Output's seq advance + RawTcp::Output's mIpId++      conn/FakeTcp.cpp:43-49, conn/RawTcp.cpp:111-121
 *   rsk_tcp_recv_ack_batch <- FakeTcp::OnRecv's ack update                                  conn/FakeTcp.cpp:52-66
 *   rsk_demux_batch       <- the per-packet conn lookups of the receive path, batched:
 *                            INetGroup::Input by connKey (conn/INetGroup.cpp:57-83), IAppGroup::Input
 *                            by cmd (conn/IAppGroup.cpp:76-96), ServerGroup::OnRecv by IdBuf
 *                            (server/ServerGroup.cpp:44-60), SubGroup::OnRecv by (dst, conv)
 *                            (server/SubGroup.cpp:31-50), ClientGroup::OnRecv by conv (client/ClientGroup.cpp:66-80)
 */
#ifndef RSK_CODEC_H
#define RSK_CODEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- wire constants (include/rstype.h:11-12, include/rscomm.h:19, conn/RConn.cpp:20) ---------- */
#define RSK_HASH_BUF_SIZE 8     /* tag bytes = last 8 bytes of the MD5 digest             */
#define RSK_ID_BUF_SIZE 8       /* IdBuf bytes                                            */
#define RSK_ENC_HEAD_SIZE 23    /* EncHead wire size: len,cmd,id[8],conv u32,key u64,rsvd */
#define RSK_HEAD_SIZE 31        /* RConn::HEAD_SIZE = 8 + 23                              */
#define RSK_MAX_PKT_SIZE 1500   /* OM_MAX_PKT_SIZE                                         */
#define RSK_MAX_PAYLOAD (RSK_MAX_PKT_SIZE - RSK_HEAD_SIZE) /* 1469                          */
#define RSK_TCPINFO_WIRE_SIZE 21 /* TcpInfo::Encode record: src,dst,sp,dp,seq,ack,flag      */

/* EncHead::TYPE (bean/EncHead.h:14-20) */
#define RSK_CMD_DATA 0
#define RSK_CMD_CONV_RST 1
#define RSK_CMD_NETCONN_RST 2
#define RSK_CMD_KEEP_ALIVE_REQ 3
#define RSK_CMD_KEEP_ALIVE_RESP 4

/* TCP flag bits as RawTcp reads them (tcp[13]) */
#define RSK_TH_FIN 0x01
#define RSK_TH_SYN 0x02
#define RSK_TH_RST 0x04
#define RSK_TH_PUSH 0x08
#define RSK_TH_ACK 0x10

/* pcap datalink types accepted by RawTcp::RawInput (RawTcp.cpp:144-165) */
#define RSK_DLT_NULL 0
#define RSK_DLT_EN10MB 1

/* ---- error codes returned by every entry point --------------------------------------------- */
#define RSK_OK 0
#define RSK_EINVAL (-22)   /* bad argument (NULL where required, n too large, bad datalink)  */
#define RSK_ENOMEM (-12)   /* device/host allocation failed                                   */
#define RSK_EDEVICE (-5)   /* a HIP runtime call failed (see rsk_last_error())                */

/* ---- per-packet status codes ---------------------------------------------------------------- */
/* Encode (RConn::Output, RConn.cpp:87-128): status[i] = 31 + P (frame length) when the frame was
 * written; RSK_SEND_OVERSIZE (-1) when 31 + P > 1500 (RConn.cpp:94-98, nothing written);
 * RSK_SEND_RESET (0) when P == 0 (the reference calls RConnReset::SendReset instead of framing,
 * RConn.cpp:119-123; nothing written, the caller sends the reset). */
#define RSK_SEND_OVERSIZE (-1)
#define RSK_SEND_RESET 0

/* Decode (RConn::OnRecv, RConn.cpp:64-85): */
#define RSK_RECV_VALID 1   /* tag verified; payload forwarded to IGroup::OnRecv (:73-75)      */
#define RSK_RECV_CLOSE 0   /* nread <= 31 on TCP with FIN|RST: NotifyTcpFinOrRst, return 0    */
#define RSK_RECV_DROP (-1) /* everything else: return -1                                      */

/* Parse (RawTcp::RawInput, RawTcp.cpp:138-237 + cap2uv :239-244): */
#define RSK_PARSE_DROP 0      /* silently dropped (reference returns 0 before delivery)       */
#define RSK_PARSE_DELIVER 1   /* handed to cap2uv -> syncInput -> RConn::OnRecv               */
#define RSK_PARSE_SYN 2       /* SYN with an ack pool: TcpAckPool::AddInfoFromPeer, return 0   */
#define RSK_PARSE_MALFORMED 3 /* header runs past cap_len, or negative payload_len with FIN|RST
                                 (the reference memcpy's a negative length there: UB,
                                 RawTcp.cpp:251) — defined here as a drop                      */
#define RSK_PARSE_SLOT_SHORT 4 /* rsk_parse_decode_slots_batch only: a byte the parse or decode
                                  reads lies past the staged slot; resubmit the packet whole   */

/* parse flags */
#define RSK_PARSE_HAS_ACK_POOL 0x1 /* RawTcp::mTcpAckPool != nullptr                          */
#define RSK_PARSE_IS_SERVER 0x2    /* RawTcp::mIsServer: SYN info is Reverse()d (:222-224)     */

/* Largest n of any batch entry point (RSK_EINVAL above it): every launch has at most one work-item
 * per packet rounded up to its 256-thread blocks, and a grid holds at most 2^32 - 1 work-items (the
 * encode copy waves -- 64 work-items per packet -- run in several launches). */
#define RSK_MAX_BATCH 0xFFFF0000u

/* ---- context -------------------------------------------------------------------------------- */
typedef struct rsk_ctx rsk_ctx;

/* Create a codec context bound to HIP device `device` for hash key `key` (host pointer, key_len
 * bytes, any length; rsock's default is "hello135", bean/RConfig.h:44).  The tag is
 * MD5(key || payload[0])[8..15] (util/rhash.cpp:20-41).  The key's MD5 message schedule is
 * precomputed here (chaining state of the whole-key blocks, the constant words of the block that
 * carries the payload byte, the padding block when one is needed), and one GPU launch (k_tag_table)
 * compresses the key's 256 possible tags into a 2-KB device table for RSK_TAG_TABLE.  The context
 * starts in RSK_TAG_MD5.  Synchronous; returns NULL on failure (rsk_last_error). */
rsk_ctx *rsk_create(const uint8_t *key, uint32_t key_len, int device);
void rsk_destroy(rsk_ctx *ctx);

/* Tag mode of every later framing / verifying launch of this context (outputs are identical):
 *   RSK_TAG_MD5    (default) one MD5 compression per packet and lane, as the reference computes it
 *                  per packet (compute_hash / hash_equal, util/rhash.cpp:20-41, 71-92);
 *   RSK_TAG_TABLE  the tag is a function of payload[0] alone, so it is looked up in the key's
 *                  256-entry table (staged in LDS per block) instead of recomputed.
 * The mode is read when a call is issued (a hipGraph keeps the mode of its capture); do not change it
 * while another thread issues calls on the same context.  rsk_set_tag_mode returns RSK_EINVAL for an
 * unknown mode, rsk_get_tag_mode the current mode (or RSK_EINVAL for a NULL ctx). */
#define RSK_TAG_MD5 0
#define RSK_TAG_TABLE 1
int rsk_set_tag_mode(rsk_ctx *ctx, int mode);
int rsk_get_tag_mode(const rsk_ctx *ctx);

/* Encode path of this context's rsk_encode_batch calls (outputs are identical):
 *   RSK_ENC_PATH_AUTO     (default) chosen per call of >= 16384 packets from the mean payload of the
 *                         context's last sampled batch (table under rsk_encode_batch);
 *   RSK_ENC_PATH_PER_SET  one kernel, 64 packets per wave (every batch shape);
 *   RSK_ENC_PATH_TWO_PASS a header pass (MD5 tags 64 to a wave, 32-B records in the stream's scratch),
 *                         then copy waves of 1, 2 or 4 packets: 4 below a mean payload of 880 B, 2 below
 *                         1160 B, 1 above (batches of long frames); below 880 B, when the sampled frames
 *                         lie back to back sharing their boundary 16-B chunks (byte-packed, no pad),
 *                         an output-stationary copy instead (waves own 2-KB blocks of the frame arena
 *                         and write each shared chunk once; frames out of packet order or more than
 *                         32 KB apart are copied packet by packet by the same launch);
 *   RSK_ENC_PATH_SHORT    the per-set kernel with every set on the flat chunk list (batches of short
 *                         frames).
 * Read when a call is issued, as the tag mode; RSK_EINVAL for an unknown path. */
#define RSK_ENC_PATH_AUTO 0
#define RSK_ENC_PATH_PER_SET 1
#define RSK_ENC_PATH_TWO_PASS 2
#define RSK_ENC_PATH_SHORT 3
int rsk_set_encode_path(rsk_ctx *ctx, int path);

/* Streams: a context may be used from several streams at once.  Its device scratch (compaction
 * ballots and look-back state, demux and send-seq tables) is kept per stream, so calls on different streams
 * never share it; calls on ONE stream must be issued in the order the caller wants them to run
 * (from one host thread at a time, as with any hipStream_t).  The only per-context state the
 * kernels read is the immutable key schedule and tag table (and the tag mode, passed by value).
 *
 * Pre-size the scratch of `stream` (rsk_reserve: the legacy default stream, NULL) for batches of up
 * to n packets: the compaction state and, for n >= 16384, the header records of the two-pass encode
 * and wire build (max(40 n + 24, 96 min(n, 2^20)) bytes: 32-B records and the output-stationary
 * copy's block map) -- only for a context that encodes: one held to RSK_ENC_PATH_TWO_PASS, or an AUTO
 * context that has already run an rsk_encode_batch call (so a decode- or demux-only context pays
 * nothing for them; a failed records allocation is not an error: eager calls allocate them on demand,
 * a captured call then takes the per-set kernel).  Batch calls grow the scratch on demand, which waits
 * for that stream to drain and allocates; reserve first if batch calls will be captured into a hipGraph. */
int rsk_reserve(rsk_ctx *ctx, uint32_t n_max);
int rsk_reserve_stream(rsk_ctx *ctx, uint32_t n_max, void *stream);
/* Scratch stays allocated per stream until the context is destroyed or the stream is released:
 * rsk_release_stream waits for `stream` to drain and frees its scratch (call it before destroying a
 * stream whose handle value a later stream may reuse).  A batch call issued while `stream` is being
 * captured into a hipGraph cannot allocate, grow or initialise that scratch (RSK_EINVAL): reserve
 * the stream and run one eager call on it before the capture.  A graph's scratch is its capture
 * stream's: replay it on that stream, or on streams ordered with it.  Graphs captured on `stream`
 * point at that scratch: destroy them before rsk_release_stream (a replay afterwards would use freed
 * device memory). */
int rsk_release_stream(rsk_ctx *ctx, void *stream);

/* Device-side error flags, sticky per context.  RSK_DEVERR_LOOKBACK: a decoupled look-back (the
 * VALID-list compaction of the decode entry points, the demux) gave up waiting for a predecessor
 * tile after ~4M polls, so that call's valid_idx / n_valid / demux outputs are wrong (a compaction
 * that gave up anywhere writes n_valid = 0xFFFFFFFF); the spin limit exists so that such a stall can
 * never hang the GPU.  rsk_check_device_errors waits for the context's streams (those it has
 * scratch on, and its shim stream; not the whole device -- except for a context with a call captured
 * into a hipGraph, whose replays may run on streams it never saw: then the whole device, until
 * rsk_forget_captures), stores the flags in *flags (may be NULL) and clears them; when any flag was
 * set it returns RSK_EDEVICE and re-initialises the context's look-back state on every stream at its
 * next call there (graphs captured earlier must be captured again). */
#define RSK_DEVERR_LOOKBACK 0x1u
/* RSK_DEVERR_TABLE: a demux key probe walked the whole key table without finding its key or a free
 * slot (the table is kept all-ones between calls, each call clearing the slots it claimed; a table
 * left dirty -- which no completed call does -- would otherwise hang the probe): that call's demux
 * outputs are wrong, and the table is filled again at the next call. */
#define RSK_DEVERR_TABLE 0x2u
int rsk_check_device_errors(rsk_ctx *ctx, uint32_t *flags);
/* The caller has destroyed every graph that captured this context's calls (or replays them only on
 * streams this context has scratch on): rsk_check_device_errors waits for the context's streams
 * again instead of the whole device. */
int rsk_forget_captures(rsk_ctx *ctx);

/* Text of the last HIP error seen by this thread (static storage). */
const char *rsk_last_error(void);

/* Library version string, e.g. "rsk 0.1 gfx950". */
const char *rsk_version(void);

/* ---- batch encode (RConn::Output framing) --------------------------------------------------- */
typedef struct rsk_encode_in {
    const uint8_t *payload_arena; /* device bytes                                           */
    const uint64_t *pay_off;      /* [n] byte offset of packet i's payload in payload_arena  */
    const uint16_t *pay_len;      /* [n] P = nread                                           */
    const uint8_t *cmd;           /* [n] EncHead cmd                                         */
    const uint32_t *conv;         /* [n] EncHead conv                                        */
    const uint64_t *conn_key;     /* [n] EncHead connKey                                     */
    const uint8_t *id;            /* [n*8] per-packet IdBuf, or NULL to use id_uniform       */
    uint8_t id_uniform[8];        /* IdBuf used for every packet when id == NULL             */
} rsk_encode_in;

typedef struct rsk_encode_out {
    uint8_t *frame_arena;     /* device bytes                                              */
    const uint64_t *frame_off;/* [n] where frame (wire packet) i starts; any offset is correct
                                 and takes the vector path (16-B aligned: no partial head chunk) */
    int32_t *status;          /* [n] 31+P, RSK_SEND_OVERSIZE or RSK_SEND_RESET              */
    uint32_t flags;           /* RSK_ENC_* below; 0 = write exactly 31+P bytes per frame      */
} rsk_encode_out;

/* RSK_ENC_ZERO_PAD16: the encoder may also write zeros from each frame's end (31+P) up to the
 * next 16-byte boundary of the arena address.  The caller asserts those bytes belong to no other
 * frame (e.g. frames in 16-B-multiple slots).  This mirrors the reference, whose frames sit in a
 * zeroed 1500-B buffer (RConn.cpp:100), and lets every 16-B chunk of a slot be written whole —
 * no byte stores and no partially written cache lines, which the memory side otherwise services
 * with read-modify-write. */
#define RSK_ENC_ZERO_PAD16 0x1u
/* RSK_ENC_ZERO_PAD128: as RSK_ENC_ZERO_PAD16 but up to the next 128-byte (cache-line) boundary;
 * takes precedence over RSK_ENC_ZERO_PAD16. */
#define RSK_ENC_ZERO_PAD128 0x2u

/* frame_i = tag(8) | EncHead(23) | payload(P), written to frame_arena + frame_off[i].
 * Frames must not overlap each other or the payload arena.
 * Three device paths, identical bytes (rsk_set_encode_path): the per-set kernel (64 packets per wave),
 * the short-frame kernel (every set on the flat chunk list) and the two-pass form (a header pass: the
 * MD5 tags 64 to a wave into 32-B records in the stream's scratch; then copy waves of 1, 2 or 4
 * packets).  AUTO chooses per call of >= 16384 packets by the mean payload of the context's last
 * sampled batch: <= 96 B short-frame, < 224 B per-set, < 400 B short-frame, < 880 B two-pass with 4
 * packets per copy wave, < 1160 B 2, else 1; smaller batches take the per-set kernel.
 * The statistic is a host-mapped word the previous calls' kernels left (read without synchronisation:
 * calls issued back to back see it late, which only delays a switch of traffic mix); the first such call
 * on a context, which has no statistic yet, samples its own batch with one 64-thread launch on
 * `stream` and waits for an event recorded behind it -- i.e. for `stream`'s work up to that launch,
 * since a stream runs in order (with this thread's capture mode relaxed for the wait); a failed
 * wait returns RSK_EDEVICE.  A call being captured, or issued on the legacy NULL stream, does not
 * wait: it takes the per-set kernel, and the sample launched behind it decides the next calls.  A call
 * captured into a hipGraph keeps the path it was captured with, and one captured on a stream without
 * reserved records takes the per-set kernel.  rsk_set_encode_path fixes the path for a context
 * (e.g. one fed alternating long- and short-frame batches). */
int rsk_encode_batch(rsk_ctx *ctx, uint32_t n, const rsk_encode_in *in, const rsk_encode_out *out,
                     void *stream);

/* ---- batch encode straight to wire packets (RConn::Output + RawTcp::SendRawTcp) ---
 * RawTcp::SendRawTcp (conn/RawTcp.cpp:280-341) hands each frame to libnet 1.1.6:
 * libnet_build_tcp(sp, dp, seq, ack, flag, win 65535, sum auto, urg 0) and
 * libnet_build_ipv4(40 + frame, tos 0, id = mIpId++, IP_DF, TTL 64, IPPROTO_TCP, sum auto, src, dst).
 * This entry point frames AND builds the packet in one pass: out->frame_arena + frame_off[i] receives
 * [eth 14 if with_eth] | IPv4 20 | TCP 20 | tag 8 | EncHead 23 | payload, with the IPv4 header checksum
 * and the TCP checksum (RFC 793 pseudo-header, RFC 1071 sum over header + frame) filled in.
 * status[i] = wire length (14? + 40 + 31 + P), RSK_SEND_OVERSIZE or RSK_SEND_RESET as for
 * rsk_encode_batch; out->flags as there (padding counts from the end of the wire packet).  The value
 * RConn::Output returns for a sent frame is SendRawTcp's `payload_len` (RawTcp.cpp:340), i.e. the
 * frame length status[i] - 40 - (with_eth ? 14 : 0).  seq and ip_id are the caller's per-packet
 * values: the reference advances them per send (FakeTcp::Output: seq += 31 + nread, FakeTcp.cpp:43-49;
 * RawTcp::Output: mIpId++, RawTcp.cpp:118-120), so one connection's batch carries
 * seq[i] = seq0 + sum_{k<i} (31 + P_k) and ip_id[i] = id0 + i.
 * Two device paths, identical bytes: the per-set wire kernels (a flat half and a per-packet half),
 * and (round 6) the two-pass form -- a header pass writing each packet's header image (80 / 96 B,
 * RAW4 / Ethernet) into the stream's scratch, then copy waves of 4 / 2 / 1 packets that sum the
 * payload into the TCP checksum -- run per chunk of 2^20 packets.  The path follows the context's
 * rsk_set_encode_path (TWO_PASS: the two-pass form; any other forced path: the per-set kernels) or,
 * under AUTO, the sampled mean payload: per-set below 160 B and for Ethernet packets from 1300 B, the
 * two-pass form otherwise, 4 packets per copy wave, RAW4 from 1080 B 2. */
typedef struct rsk_wire_in {
    const uint32_t *src, *dst; /* [n] TcpInfo::src / dst: IPv4 addresses as stored (network order) */
    const uint16_t *sp, *dp;   /* [n] ports, host order                                           */
    const uint32_t *seq, *ack; /* [n] host order (TcpInfo seq / ack at send time)                 */
    const uint8_t *flag;       /* [n] TCP flags (TcpInfo::flag)                                   */
    const uint16_t *ip_id;     /* [n] IPv4 identification (RawTcp::mIpId++, host order)           */
    uint8_t eth[14];           /* link header written before the IPv4 header when with_eth       */
    uint8_t with_eth;          /* 0: LIBNET_RAW4 layout (IPv4 first); 1: Ethernet frame           */
} rsk_wire_in;
int rsk_encode_wire_batch(rsk_ctx *ctx, uint32_t n, const rsk_encode_in *in, const rsk_wire_in *wire,
                          const rsk_encode_out *out, void *stream);

/* ---- batch decode + verify (RConn::OnRecv) --------------------------------------------------- */
typedef struct rsk_decode_out {
    uint8_t *hlen;       /* [n] EncHead len byte as received (payload starts at 8 + hlen)      */
    uint8_t *cmd;        /* [n]                                                               */
    uint8_t *id;         /* [n*8]                                                             */
    uint32_t *conv;      /* [n]                                                               */
    uint64_t *conn_key;  /* [n]                                                               */
    uint16_t *pay_off;   /* [n] payload offset relative to the frame start (= 8 + hlen)       */
    uint16_t *pay_len;   /* [n] nread - 8 - hlen                                              */
    int8_t *status;      /* [n] RSK_RECV_*                                                    */
    uint32_t *valid_idx; /* [n] order-stable list of i with status == RSK_RECV_VALID (may be NULL) */
    uint32_t *n_valid;   /* [1] number of entries in valid_idx (device; may be NULL)            */
} rsk_decode_out;
/* For packets whose status is not RSK_RECV_VALID, hlen/cmd/id/conv/conn_key/pay_off/pay_len are
 * written as zero (the reference never exposes fields of a dropped frame). */

/* frame i = frame_len[i] bytes at frame_arena + frame_off[i]; is_tcp_close[i] != 0 marks a frame
 * that arrived on fake TCP with FIN or RST set (TcpInfo::HasCloseFlag, bean/TcpInfo.h:31); NULL
 * means "UDP / no close flag" for all packets. */
int rsk_decode_batch(rsk_ctx *ctx, uint32_t n, const uint8_t *frame_arena, const uint64_t *frame_off,
                     const uint16_t *frame_len, const uint8_t *is_tcp_close, const rsk_decode_out *out,
                     void *stream);

/* ---- header-only batches (host-resident deployments) ------------------------------------------
 * The codec reads one payload byte per frame (payload[0] for the tag) and writes / verifies the
 * first 31 frame bytes: a caller whose payloads live in host memory ships only those bytes over PCIe
 * and keeps the payload where it is (assembling frame = header(31) | payload with an iovec, or the
 * memcpy RConn.cpp:104 does anyway).  Slots are 32 B, 16-B aligned, slot i at hdr + 32 i. */
typedef struct rsk_encode_hdr_in {
    const uint8_t *first_byte; /* [n] payload[0] (read only when 1 <= pay_len <= 1469)             */
    const uint16_t *pay_len;   /* [n]                                                              */
    const uint8_t *cmd;
    const uint32_t *conv;
    const uint64_t *conn_key;
    const uint8_t *id;         /* [n*8] 8-B aligned, or NULL (then id_uniform)                     */
    uint8_t id_uniform[8];
} rsk_encode_hdr_in;
/* slot i = frame bytes [0, 32): tag | EncHead | payload[0]; zero when status[i] <= 0.  status as
 * rsk_encode_batch. */
int rsk_encode_headers_batch(rsk_ctx *ctx, uint32_t n, const rsk_encode_hdr_in *in, uint8_t *hdr,
                             int32_t *status, void *stream);
/* slot i = frame bytes [0, 31) and, in byte 31, the byte OnRecv hashes: frame[8 + len] with
 * len = frame[8] (= frame[31] for a well-formed frame); rsk_stage_decode_header builds it.
 * frame_len[i] is the frame's full length; outputs exactly as rsk_decode_batch on the whole frame. */
int rsk_decode_headers_batch(rsk_ctx *ctx, uint32_t n, const uint8_t *hdr, const uint16_t *frame_len,
                             const uint8_t *is_tcp_close, const rsk_decode_out *out, void *stream);
/* Host: the decode slot of one received frame (host pointers). */
void rsk_stage_decode_header(const uint8_t *frame, int nread, uint8_t *slot);
/* Host batch forms (host pointers; nthreads <= 1 runs on the caller's thread): stage the slots of n
 * frames at arena + frame_off[i]; assemble frame i = hdr slot bytes [0, 31) | payload (status[i] - 31
 * bytes at payload_arena + pay_off[i]) for status[i] > 0 — the copy RConn::Output makes
 * (RConn.cpp:100-104) when the sender needs one contiguous frame. */
int rsk_stage_decode_headers(uint32_t n, const uint8_t *arena, const uint64_t *frame_off,
                             const uint16_t *frame_len, uint8_t *slots, int nthreads);
int rsk_assemble_frames(uint32_t n, const uint8_t *hdr, const int32_t *status, const uint8_t *payload_arena,
                        const uint64_t *pay_off, uint8_t *frame_arena, const uint64_t *frame_off, int nthreads);

/* ---- fused pcap parse + decode (RawTcp::RawInput -> cap2uv -> RConn::OnRecv) ----------------- */
typedef struct rsk_tcpinfo_out {
    uint32_t *src;  /* [n] ip_dst as stored (network byte order bytes, read LE) — "self" view   */
    uint32_t *dst;  /* [n] ip_src as stored                                                    */
    uint16_t *sp;   /* [n] ntohs(th_dport)                                                     */
    uint16_t *dp;   /* [n] ntohs(th_sport)                                                     */
    uint32_t *seq;  /* [n] ntohl(th_seq) (+ payload_len when delivered)                        */
    uint32_t *ack;  /* [n] ntohl(th_ack)                                                       */
    uint8_t *flag;  /* [n] th_flags                                                            */
    int8_t *parse_status; /* [n] RSK_PARSE_*                                                   */
    uint16_t *cap_pay_off; /* [n] payload (= frame) offset inside the captured packet          */
    uint16_t *cap_pay_len; /* [n] payload_len (0 unless delivered)                             */
} rsk_tcpinfo_out;
/* TcpInfo fields are written for RSK_PARSE_DELIVER and RSK_PARSE_SYN, zero otherwise.  The decode
 * outputs (`dec`) follow rsk_decode_batch on the delivered payload with is_tcp_close = flag &
 * (FIN|RST); packets that were not delivered get dec->status = RSK_RECV_DROP and zero fields. */
int rsk_parse_decode_batch(rsk_ctx *ctx, uint32_t n, const uint8_t *cap_arena, const uint64_t *cap_off,
                           const uint32_t *wire_len, const uint32_t *cap_len, int datalink, int flags,
                           const rsk_tcpinfo_out *tcp, const rsk_decode_out *dec, void *stream);

/* Host-resident capture (copy only the first ~86 B of each captured packet, keep the
 * payloads host-side): packet i's first min(cap_len[i], slot) bytes at slots + slot * i (slot a
 * multiple of 16, >= RSK_CAP_SLOT_MIN; slots 16-B aligned), staged by rsk_stage_capture_slots.  Same
 * outputs as rsk_parse_decode_batch on the whole capture (decisions use the real cap_len), except
 * that a packet whose parse or decode must read a byte past its slot (IP/TCP options, an EncHead
 * len byte that moves the hashed byte) gets parse_status RSK_PARSE_SLOT_SHORT with zero outputs
 * and dec->status RSK_RECV_DROP: resubmit those through rsk_parse_decode_batch.  With slot = 96 a
 * rsock packet (IHL 5, data offset 5, len 23) needs 86 B (EN10MB) or 76 B (NULL). */
#define RSK_CAP_SLOT_MIN 64
int rsk_parse_decode_slots_batch(rsk_ctx *ctx, uint32_t n, const uint8_t *slots, uint32_t slot,
                                 const uint32_t *wire_len, const uint32_t *cap_len, int datalink, int flags,
                                 const rsk_tcpinfo_out *tcp, const rsk_decode_out *dec, void *stream);
/* Host: stage the slots of n captured packets at arena + cap_off[i] (first min(cap_len[i], slot)
 * bytes, the rest of the slot zeroed). */
int rsk_stage_capture_slots(uint32_t n, const uint8_t *arena, const uint64_t *cap_off, const uint32_t *cap_len,
                            uint32_t slot, uint8_t *slots, int nthreads);

/* ---- TcpInfo hand-off records (cap2uv's 21-B TcpInfo::Encode) ---------------- */
/* rec[21*i ..] = src LE32 | dst LE32 | sp LE16 | dp LE16 | seq LE32 | ack LE32 | flag. */
int rsk_tcpinfo_encode_batch(rsk_ctx *ctx, uint32_t n, const uint32_t *src, const uint32_t *dst,
                             const uint16_t *sp, const uint16_t *dp, const uint32_t *seq,
                             const uint32_t *ack, const uint8_t *flag, uint8_t *rec, void *stream);
/* The consumer side (RawTcp::syncInput, conn/RawTcp.cpp:262-276 -> TcpInfo::Decode,
 * bean/TcpInfo.cpp:35-47 -> RConn::OnRecv): record i = nread[i] bytes at rec_arena + rec_off[i], a
 * 21-B TcpInfo record followed by the frame (what cap2uv sends, RawTcp.cpp:239-260).  A record of
 * nread >= 21 bytes gets parse_status RSK_PARSE_DELIVER, its TcpInfo fields, cap_pay_off 21,
 * cap_pay_len nread - 21, and dec = rsk_decode_batch on the frame with is_tcp_close = flag &
 * (FIN|RST).  nread < 21: RSK_PARSE_DROP, zero TcpInfo, dec->status RSK_RECV_DROP (syncInput
 * returns before Input for nread <= 0 and for a failed Decode; for 12 <= nread < 21 the reference's
 * Decode does not fail but reads its receive buffer past nread — TcpInfo.cpp:40 compares the
 * bytes consumed, not those left — so this is the one deliberate deviation, on malformed input). */
int rsk_syncinput_decode_batch(rsk_ctx *ctx, uint32_t n, const uint8_t *rec_arena, const uint64_t *rec_off,
                               const int32_t *nread, const rsk_tcpinfo_out *tcp, const rsk_decode_out *dec,
                               void *stream);

/* ---- fake-TCP connection state on either side of the codec --------------------------------------- */
/* Send: FakeTcp::Output (conn/FakeTcp.cpp:43-49) advances its connection's seq by
 * RConn::HEAD_SIZE + nread after every frame RConn::Output produced, and RawTcp::Output
 * (conn/RawTcp.cpp:111-121) stamps every packet it sends with mIpId++.  For a batch sent in order,
 * packet i of connection conn[i] with rsk_encode_batch's status[i] (31 + P when framed):
 *   framed (status > 0): ip_id[i] = *ip_id_next, then ++*ip_id_next (wraps at 2^16); and when
 *       conn[i] < n_conn: seq[i] = conn_seq[conn[i]], then conn_seq[conn[i]] += status[i] (mod 2^32)
 *   otherwise, or conn[i] >= n_conn: seq[i] = 0 (ip_id[i] = 0 when not framed)
 * conn_seq [n_conn] and ip_id_next [1] are device state updated in place; seq / ip_id are what
 * rsk_encode_wire_batch takes.  n <= 2^30.  Workspace: n_conn < 2048 takes a per-tile connection table
 * (<= 4 B per packet); wider n_conn the demux group-by (its workspace plus ~35 B per packet). */
int rsk_tcp_send_seq_batch(rsk_ctx *ctx, uint32_t n, const uint32_t *conn, const int32_t *status,
                           uint32_t n_conn, uint32_t *conn_seq, uint16_t *ip_id_next, uint32_t *seq,
                           uint16_t *ip_id, void *stream);
/* Receive: FakeTcp::OnRecv (conn/FakeTcp.cpp:52-66) raises its connection's ack to a delivered
 * packet's TcpInfo seq (rsk_parse_decode_batch's tcp->seq) when that is larger (unsigned compare,
 * as the reference), so over a batch conn_ack[c] = max(conn_ack[c], seq[i] of every packet i with
 * delivered[i] != 0 and conn[i] == c) — independent of order; conn[i] >= n_conn is skipped.
 * n <= 2^30 (RSK_EINVAL above). */
int rsk_tcp_recv_ack_batch(rsk_ctx *ctx, uint32_t n, const uint32_t *conn, const uint8_t *delivered,
                           const uint32_t *seq, uint32_t n_conn, uint32_t *conn_ack, void *stream);

/* ---- receive demux: stable group-by of the VALID packets on decoded fields --- */
/* The reference routes every VALID packet on its own: a map lookup per packet on the fields below,
 * packets delivered in arrival order.  rsk_demux_batch groups a decoded batch so the host does one
 * lookup per segment and hands each conn its packets as one run:
 *   - the key is the tuple of the fields selected in `fields` (unselected fields are ignored);
 *   - with RSK_DEMUX_CMD_BARRIER, a packet whose cmd != RSK_CMD_DATA (RST / keepalive, handled by
 *     IAppGroup outside the conn maps) is a segment of its own and an ordering barrier: DATA
 *     packets on either side of it never share a segment;
 *   - with RSK_DEMUX_GROUP_BARRIER instead (requires RSK_DEMUX_ID, excludes CMD_BARRIER), a control
 *     packet is a segment of its own and a barrier for the packets of its own IdBuf only: DATA
 *     packets of one IdBuf on either side of it never share a segment, packets of other IdBufs
 *     are not split by it.  That is the server's routing: ServerGroup::OnRecv (server/
 *     ServerGroup.cpp:44-60) hands each packet to its IdBuf's SubGroup, whose conns and control
 *     handling never see another IdBuf's packets, so only the order inside one IdBuf is
 *     observable.  A server batch then has about one segment per conn and epoch of its own group
 *     instead of one per conn and epoch of the whole batch;
 *   - segments are ordered by their first packet, packets inside a segment by arrival.
 * Delivering segment by segment therefore hands every conn the same packet sequence as the
 * reference's per-packet loop, and creates new conns in the same order (first occurrence). */
#define RSK_DEMUX_ID            0x01u /* EncHead IdBuf (8 B)                                      */
#define RSK_DEMUX_CONN_KEY      0x02u /* EncHead connKey                                          */
#define RSK_DEMUX_CONV          0x04u /* EncHead conv                                             */
#define RSK_DEMUX_DST           0x08u /* TcpInfo dst (SubGroup keys on BuildConvKey(dst, conv))   */
#define RSK_DEMUX_CMD_BARRIER   0x10u
#define RSK_DEMUX_GROUP_BARRIER 0x20u
typedef struct rsk_demux_in {
    const int8_t *status;      /* [n] packet i takes part iff status[i] == RSK_RECV_VALID       */
    const uint8_t *cmd;        /* [n]                                                           */
    const uint8_t *id;         /* [n*8] (8-B aligned); may be NULL unless RSK_DEMUX_ID           */
    const uint32_t *conv;      /* [n]; may be NULL unless RSK_DEMUX_CONV                         */
    const uint64_t *conn_key;  /* [n]; may be NULL unless RSK_DEMUX_CONN_KEY                     */
    const uint32_t *dst;       /* [n]; may be NULL unless RSK_DEMUX_DST                          */
} rsk_demux_in;
typedef struct rsk_demux_out {
    uint32_t *perm;      /* [n] packet indices, segment by segment (first n_valid entries used)   */
    uint32_t *seg_off;   /* [n+1] segment s = perm[seg_off[s] .. seg_off[s+1]) (first n_seg+1)   */
    uint32_t *seg_first; /* [n] first packet of segment s (its key representative), increasing    */
    uint32_t *n_seg;     /* [1]                                                                   */
    uint32_t *n_valid;   /* [1]                                                                   */
} rsk_demux_out;
/* n <= 2^30.  Workspace (per stream, grown on demand): about 75 B per packet.  GROUP_BARRIER runs
 * two group-bys (the control packets by IdBuf, then every packet by the key with each DATA packet's
 * epoch inside its IdBuf), writing
 * the first one's result to `out` before the second overwrites it. */
int rsk_demux_batch(rsk_ctx *ctx, uint32_t n, const rsk_demux_in *in, uint32_t fields,
                    const rsk_demux_out *out, void *stream);

/* ---- capture filter ------------------------------------------------------- */
/* RCap::doInit (cap/RCap.cpp:64-88) compiles BuildFilterStr("tcp", srcIp, dstIp, srcPorts, dstPorts,
 * isServer) (cap/cap_util.cpp:67-144) into the kernel's BPF filter.  For a client that string is
 *   F  = tcp [and (ip src S)] [and (ip dst D)] [and ( src port p or ... src portrange a-b ... )]
 *        [and ( dst port p or ... dst portrange a-b ... )]
 * and for a server  ((tcp[tcpflags] & tcp-syn != 0) and F') or (F and (tcp[tcpflags] & (tcp-syn) == 0))
 * where F' is F with every "dst" replaced by "src".  rsk_capture_filter_batch evaluates that
 * predicate with libpcap's meaning of each primitive:
 *   tcp          IPv4 with protocol 6, or IPv6 with next header 6 (directly, or after a fragment
 *                header, 44);
 *   ip src/dst   IPv4 only, the address field equals S / D;
 *   [src|dst] port / portrange   IPv4 with protocol 6, 17 or 132 and fragment offset 0, or IPv6
 *                with next header 6, 17 or 132; the port field (at 4 * IHL on IPv4, 40 on IPv6)
 *                equals p / lies in [a, b];
 *   tcp[tcpflags]  IPv4 with protocol 6 and fragment offset 0: TCP header byte 13.
 * Link layer: DLT_EN10MB ethertype 0x0800 / 0x86dd at bytes 12-13; DLT_NULL a 4-byte family in
 * host order, 2 = IPv4, 24 / 28 / 30 = IPv6 (BSD values).  Evaluation is left to right with
 * short-circuit; a field read past cap_len rejects the packet (as a BPF load out of bounds does).
 * match[i] = 1 / 0; match_idx / n_match (optional, may be NULL) list the matches in order. */
#define RSK_FILTER_MAX_PORTS 64
typedef struct rsk_port_list {
    uint16_t n_single, n_range;            /* RPortList::GetSinglePortList / GetPortRangeList sizes */
    uint16_t single[RSK_FILTER_MAX_PORTS]; /* in list order                                        */
    uint16_t range[RSK_FILTER_MAX_PORTS][2]; /* [source, dest], source < dest (RPortList.cpp:21-27) */
} rsk_port_list;
typedef struct rsk_capture_filter {
    uint32_t src_ip, dst_ip;  /* IPv4 as stored in the header (network-order bytes read LE)        */
    uint8_t has_src_ip;       /* srcIp non-empty                                                  */
    uint8_t has_dst_ip;       /* dstIp non-empty                                                  */
    uint8_t is_server;
    uint8_t reserved;         /* 0                                                                */
    rsk_port_list src_ports, dst_ports;
} rsk_capture_filter;
int rsk_capture_filter_batch(rsk_ctx *ctx, uint32_t n, const uint8_t *cap_arena, const uint64_t *cap_off,
                             const uint32_t *cap_len, int datalink, const rsk_capture_filter *filter,
                             uint8_t *match, uint32_t *match_idx, uint32_t *n_match, void *stream);
/* The filter and rsk_parse_decode_batch in one pass over a capture batch (the parse reuses the
 * filter's header window): match[i] as above; a packet the filter passes gets exactly
 * rsk_parse_decode_batch's outputs, one it rejects (pcap never hands it to RawTcp::RawInput) gets
 * parse_status RSK_PARSE_DROP, zero TcpInfo and dec->status RSK_RECV_DROP; dec->valid_idx lists the
 * VALID packets in order. */
int rsk_filter_parse_decode_batch(rsk_ctx *ctx, uint32_t n, const uint8_t *cap_arena, const uint64_t *cap_off,
                                  const uint32_t *wire_len, const uint32_t *cap_len, int datalink, int flags,
                                  const rsk_capture_filter *filter, uint8_t *match, const rsk_tcpinfo_out *tcp,
                                  const rsk_decode_out *dec, void *stream);
/* Host: the exact string BuildFilterStr returns for this filter (proto "tcp", addresses dotted),
 * NUL-terminated into buf.  Returns its length, or -1 if buf_len is too small. */
int rsk_filter_str(const rsk_capture_filter *filter, char *buf, size_t buf_len);

/* ---- single-packet shims with the reference signatures (host pointers) ----------------------- */
/* These run the same HIP kernels on a batch of one (device round trip, synchronous), so a caller
 * can swap them in per call.  They are a compatibility surface, not a fast path. */
/* Writes the 8-byte tag for data[0] to tag_out; returns tag_out + 8 (NULL if data_len <= 0). */
uint8_t *rsk_compute_hash(rsk_ctx *ctx, uint8_t *tag_out, const uint8_t *data, int data_len);
/* 1 if tag == MD5(key || data[0])[8..15], 0 otherwise (0 when data == NULL or data_len <= 0). */
int rsk_hash_equal(rsk_ctx *ctx, const uint8_t *tag, const uint8_t *data, int data_len);
/* Writes the 23-byte EncHead; returns p + 23, or NULL when p == NULL or buf_len < 23. */
uint8_t *rsk_enchead_enc2buf(rsk_ctx *ctx, uint8_t *p, int buf_len, uint8_t cmd, const uint8_t id[8],
                             uint32_t conv, uint64_t conn_key);
/* Decodes fields; returns p + len (len = p[0]), or NULL when p == NULL, buf_len < 23 or len > buf_len.
 * Any output pointer may be NULL. */
const uint8_t *rsk_enchead_decodebuf(rsk_ctx *ctx, const uint8_t *p, int buf_len, uint8_t *len,
                                     uint8_t *cmd, uint8_t id[8], uint32_t *conv, uint64_t *conn_key);

/* ---- connKey helpers (host, pure integer arithmetic) ---------------------------------------- */
/* KeyForTcp: 0x10000000 | (dp << 16) | sp — the type bit overlaps dp bit 12, reproduced as-is. */
uint64_t rsk_key_for_tcp(uint16_t sp, uint16_t dp);
uint64_t rsk_key_for_udp(uint16_t sp, uint16_t dp);

/* ---- synthetic workload generator (device; used by bench/tests, not by the codec) ------------ */
/* Fills n bytes at dst with the splitmix64 stream: 8-byte word w = splitmix64(seed + w) (LE). */
int rsk_fill_splitmix(void *dst, uint64_t nbytes, uint64_t seed, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* RSK_CODEC_H */
