/*
 * rsk_rconn.h — C ABI of the RConn-shaped batching adapter (rsock_amd/csrc/rconn_gpu.h).
 *
 * Replaces the per-packet surface of RConn (conn/RConn.h:34-37): rsk_rconn_output mirrors
 * RConn::Output (conn/RConn.cpp:87-128) and rsk_rconn_onrecv mirrors RConn::OnRecv
 * (conn/RConn.cpp:64-85), with the same return values, but the framing / verification runs in
 * batches on the GPU through include/rsk_codec.h.  Results are delivered, in input order, through
 * the callbacks when a batch completes (batch full, or rsk_rconn_flush).
 *
 * Buffers passed to output/onrecv are copied before the call returns (the reference's rbuf_t is a
 * non-owning view valid only during the call, rsutil.h:56-58).  Frame and payload pointers handed to
 * the callbacks are valid only during the callback.  Not thread-safe: one adapter per loop thread,
 * like RConn.
 */
#ifndef RSK_RCONN_H
#define RSK_RCONN_H

#include <stdint.h>

#include "rsk_codec.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rsk_rconn rsk_rconn;

/* RawTcp::Send / BtmUdpConn::Send: one framed packet (tag | EncHead | payload), len = 31 + P */
typedef int (*rsk_send_fn)(const char *frame, int len, void *user, void *cb_arg);
/* RConnReset::SendReset: Output with nread == 0 */
typedef int (*rsk_reset_fn)(void *user, void *cb_arg);
/* IGroup::OnRecv (status RSK_RECV_VALID: payload = frame + 8 + hlen, payload_len = nread - 8 - hlen),
 * NetService::NotifyTcpFinOrRst (RSK_RECV_CLOSE) or a drop (RSK_RECV_DROP, fields zero). */
typedef int (*rsk_recv_fn)(int status, uint8_t hlen, uint8_t cmd, const uint8_t *id, uint32_t conv,
                           uint64_t conn_key, const char *payload, int payload_len, void *user, void *cb_arg);

/* batch = packets per GPU batch (double-buffered); NULL on failure (see rsk_last_error()). */
rsk_rconn *rsk_rconn_create(const uint8_t *key, uint32_t key_len, int device, uint32_t batch);
void rsk_rconn_destroy(rsk_rconn *r); /* flushes first */
void rsk_rconn_set_callbacks(rsk_rconn *r, rsk_send_fn send, rsk_reset_fn reset, rsk_recv_fn recv,
                             void *cb_arg);

/* RConn::Output: nread < 0 -> nread; 31 + nread > 1500 -> -1; otherwise the packet is queued and
 * 31 + nread is returned.  nread == 0 (RConnReset::SendReset, RConn.cpp:119-123) is queued too and
 * returns 0: its reset callback fires at delivery, after the send callbacks of every packet queued
 * before it and before those queued after it (send and reset callbacks come in input order). */
int rsk_rconn_output(rsk_rconn *r, int64_t nread, const char *base, uint8_t cmd, const uint8_t id[8],
                     uint32_t conv, uint64_t conn_key, void *user);
/* RConn::OnRecv: queues the frame (tcp_close = TcpInfo::HasCloseFlag on a TCP frame); returns 0 or
 * RSK_E*; the per-frame status arrives in the recv callback. */
int rsk_rconn_onrecv(rsk_rconn *r, int64_t nread, const char *base, int tcp_close, void *user);
/* Run everything queued and deliver every outstanding result. */
int rsk_rconn_flush(rsk_rconn *r);
/* Send and reset callbacks run at delivery, not inside rsk_rconn_output, so their return values
 * (RawTcp::Send / RConnReset::SendReset results, which RConn::Output returns synchronously,
 * RConn.cpp:108-123) cannot be the output call's result: every callback that returned < 0 is
 * counted here instead (since creation). */
uint64_t rsk_rconn_callback_failures(const rsk_rconn *r);

#ifdef __cplusplus
}
#endif
#endif /* RSK_RCONN_H */
