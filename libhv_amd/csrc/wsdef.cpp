// wsdef.cpp -- libhv's wsdef.c helpers (reference http/wsdef.c:11-46).
// The handshake digest (RFC 6455 sec. 4.2.2: base64(SHA-1(key + GUID))) is
// per-connection host work; frame building masks its payload on the GPU via
// websocket_build_frame.
#include "wsdef.h"

#include <stdint.h>
#include <string.h>

#include "websocket_parser.h"

namespace {

inline uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

// FIPS 180-4 SHA-1, one-shot over a byte string.
void sha1(const uint8_t* msg, size_t n, uint8_t out[20]) {
    uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    const uint64_t bits = (uint64_t)n * 8u;
    const size_t total = ((n + 8) / 64 + 1) * 64;
    for (size_t blk = 0; blk < total; blk += 64) {
        uint8_t b[64];
        for (size_t i = 0; i < 64; ++i) {
            const size_t k = blk + i;
            if (k < n) b[i] = msg[k];
            else if (k == n) b[i] = 0x80;
            else if (k >= total - 8) b[i] = (uint8_t)(bits >> (8 * (total - 1 - k)));
            else b[i] = 0;
        }
        uint32_t w[80];
        for (int t = 0; t < 16; ++t)
            w[t] = (uint32_t)b[4 * t] << 24 | (uint32_t)b[4 * t + 1] << 16 | (uint32_t)b[4 * t + 2] << 8 | b[4 * t + 3];
        for (int t = 16; t < 80; ++t) w[t] = rol(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1);
        uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4];
        for (int t = 0; t < 80; ++t) {
            uint32_t f, k;
            if (t < 20) { f = (bb & c) | (~bb & d); k = 0x5A827999u; }
            else if (t < 40) { f = bb ^ c ^ d; k = 0x6ED9EBA1u; }
            else if (t < 60) { f = (bb & c) | (bb & d) | (c & d); k = 0x8F1BBCDCu; }
            else { f = bb ^ c ^ d; k = 0xCA62C1D6u; }
            const uint32_t tmp = rol(a, 5) + f + e + k + w[t];
            e = d;
            d = c;
            c = rol(bb, 30);
            bb = a;
            a = tmp;
        }
        h[0] += a; h[1] += bb; h[2] += c; h[3] += d; h[4] += e;
    }
    for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 4; ++j) out[4 * i + j] = (uint8_t)(h[i] >> (24 - 8 * j));
}

int base64(const uint8_t* in, size_t n, char* out) {
    static const char tbl[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    size_t o = 0;
    for (size_t i = 0; i < n; i += 3) {
        uint32_t v = (uint32_t)in[i] << 16;
        if (i + 1 < n) v |= (uint32_t)in[i + 1] << 8;
        if (i + 2 < n) v |= in[i + 2];
        out[o++] = tbl[(v >> 18) & 63];
        out[o++] = tbl[(v >> 12) & 63];
        out[o++] = i + 1 < n ? tbl[(v >> 6) & 63] : '=';
        out[o++] = i + 2 < n ? tbl[v & 63] : '=';
    }
    // No terminator, like hv_base64_encode: ws_encode_key writes exactly 28
    // bytes and its callers pass zeroed 32-byte buffers (HttpHandler.cpp:986).
    return (int)o;
}

}  // namespace

extern "C" {

void ws_encode_key(const char* key, char accept[]) {
    static const char guid[] = WEBSOCKET_UUID;
    const size_t kn = strlen(key), gn = sizeof(guid) - 1;
    uint8_t buf[256];
    uint8_t* m = buf;
    uint8_t* heap = nullptr;
    if (kn + gn > sizeof(buf)) m = heap = new uint8_t[kn + gn];
    memcpy(m, key, kn);
    memcpy(m + kn, guid, gn);
    uint8_t digest[20];
    sha1(m, kn + gn, digest);
    delete[] heap;
    base64(digest, 20, accept);
}

int ws_calc_frame_size(int data_len, bool has_mask) {
    int size = data_len + 2;
    if (data_len >= 126) size += data_len > 0xFFFF ? 8 : 2;
    if (has_mask) size += 4;
    return size;
}

int ws_build_frame(char* out, const char* data, int data_len, const char mask[4], bool has_mask,
                   enum ws_opcode opcode, bool fin) {
    int flags = opcode;
    if (fin) flags |= WS_FIN;
    if (has_mask) flags |= WS_HAS_MASK;
    return (int)websocket_build_frame(out, (websocket_flags)flags, mask, data, (size_t)data_len);
}

}  // extern "C"
