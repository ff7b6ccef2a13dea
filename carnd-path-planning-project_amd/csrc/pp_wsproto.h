// pp_wsproto.h — the RFC 6455 subset the simulator shim speaks (pp_server.cpp): the HTTP upgrade
// (Sec-WebSocket-Accept = base64(SHA-1(key + GUID))), frame parsing of masked / unmasked client
// frames, fragmented text messages, ping -> pong, close -> close; server frames out. Header-only so
// the sanitizer driver (tests/sanitize/fuzz_host.cpp) runs the same code on malformed input. Every
// buffer a peer controls is bounded: the request head (16 KiB), one frame (64 MiB), a fragmented
// message (64 MiB) and the queue of complete messages (kMaxQueued); beyond any bound the
// connection is closed.
#pragma once
#include <ctype.h>
#include <stdint.h>
#include <string.h>

#include <deque>
#include <string>

namespace ppws {

constexpr size_t kMaxHead = 16384;
constexpr uint64_t kMaxFrame = 64u << 20;
constexpr size_t kMaxMessage = 64u << 20;
constexpr size_t kMaxQueued = 4096;

// ---- SHA-1 (FIPS 180-4) + base64: the handshake's accept key ----------------------------------
struct Sha1 {
    uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    static uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
    void block(const uint8_t* p) {
        uint32_t w[80];
        for (int i = 0; i < 16; i++) w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
        for (int i = 16; i < 80; i++) w[i] = rol(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
        for (int i = 0; i < 80; i++) {
            uint32_t f, k;
            if (i < 20) { f = (b & c) | (~b & d); k = 0x5A827999u; }
            else if (i < 40) { f = b ^ c ^ d; k = 0x6ED9EBA1u; }
            else if (i < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8F1BBCDCu; }
            else { f = b ^ c ^ d; k = 0xCA62C1D6u; }
            const uint32_t t = rol(a, 5) + f + e + k + w[i];
            e = d; d = c; c = rol(b, 30); b = a; a = t;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
    }
    void digest(const std::string& m, uint8_t out[20]) {
        std::string p = m;
        const uint64_t bits = (uint64_t)m.size() * 8;
        p += (char)0x80;
        while (p.size() % 64 != 56) p += (char)0;
        for (int i = 7; i >= 0; i--) p += (char)((bits >> (8 * i)) & 0xFF);
        for (size_t i = 0; i < p.size(); i += 64) block((const uint8_t*)p.data() + i);
        for (int i = 0; i < 5; i++)
            for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(h[i] >> (24 - 8 * j));
    }
};

inline std::string base64(const uint8_t* d, size_t n) {
    static const char* T = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    std::string o;
    for (size_t i = 0; i < n; i += 3) {
        uint32_t v = (uint32_t)d[i] << 16 | (i + 1 < n ? (uint32_t)d[i + 1] << 8 : 0) | (i + 2 < n ? d[i + 2] : 0);
        o += T[(v >> 18) & 63];
        o += T[(v >> 12) & 63];
        o += i + 1 < n ? T[(v >> 6) & 63] : '=';
        o += i + 2 < n ? T[v & 63] : '=';
    }
    return o;
}

inline std::string ws_accept(const std::string& key) {
    uint8_t dg[20];
    Sha1 s;
    s.digest(key + "258EAFA5-E914-47DA-95CA-C5AB0DC85B11", dg);
    return base64(dg, 20);
}

inline void ws_frame(std::string& out, int opcode, const char* p, size_t n) {
    out += (char)(0x80 | opcode);
    if (n < 126) out += (char)n;
    else if (n < 65536) { out += (char)126; out += (char)(n >> 8); out += (char)(n & 0xFF); }
    else { out += (char)127; for (int i = 7; i >= 0; i--) out += (char)((uint64_t)n >> (8 * i) & 0xFF); }
    out.append(p, n);
}

struct WsConn {
    int fd = -1;
    bool upgraded = false;
    bool closing = false;
    std::string in, out, frag;
    int frag_op = 0;
    std::deque<std::string> msgs;   // complete text messages, in order
};

// HTTP upgrade; false = not complete yet; sets c.closing on a bad request
inline bool handshake(WsConn& c) {
    const size_t e = c.in.find("\r\n\r\n");
    if (e == std::string::npos) { if (c.in.size() > kMaxHead) c.closing = true; return false; }
    std::string req = c.in.substr(0, e);
    c.in.erase(0, e + 4);
    std::string key;
    size_t p = 0;
    while (p < req.size()) {
        size_t q = req.find("\r\n", p);
        if (q == std::string::npos) q = req.size();
        std::string line = req.substr(p, q - p);
        const size_t col = line.find(':');
        if (col != std::string::npos) {
            std::string name = line.substr(0, col);
            for (char& ch : name) ch = (char)tolower((unsigned char)ch);
            if (name == "sec-websocket-key") {
                size_t a = col + 1;
                while (a < line.size() && line[a] == ' ') a++;
                size_t b = line.size();
                while (b > a && (line[b - 1] == ' ' || line[b - 1] == '\r')) b--;
                key = line.substr(a, b - a);
            }
        }
        p = q + 2;
    }
    if (key.empty()) {
        c.out += "HTTP/1.1 400 Bad Request\r\nContent-Length: 0\r\nConnection: close\r\n\r\n";
        c.closing = true;
        return false;
    }
    c.out += "HTTP/1.1 101 Switching Protocols\r\nUpgrade: websocket\r\nConnection: Upgrade\r\nSec-WebSocket-Accept: " +
             ws_accept(key) + "\r\n\r\n";
    c.upgraded = true;
    return true;
}

// parse complete frames from c.in
inline void ws_read(WsConn& c) {
    for (;;) {
        const size_t n = c.in.size();
        if (n < 2) return;
        const uint8_t* b = (const uint8_t*)c.in.data();
        const bool fin = b[0] & 0x80;
        const int op = b[0] & 0x0F;
        const bool masked = b[1] & 0x80;
        uint64_t len = b[1] & 0x7F;
        size_t h = 2;
        if (len == 126) { if (n < 4) return; len = (uint64_t)b[2] << 8 | b[3]; h = 4; }
        else if (len == 127) { if (n < 10) return; len = 0; for (int i = 0; i < 8; i++) len = len << 8 | b[2 + i]; h = 10; }
        if (len > kMaxFrame) { c.closing = true; return; }
        const size_t mh = masked ? 4 : 0;
        if (n < h + mh + len) return;
        std::string pay = c.in.substr(h + mh, (size_t)len);
        if (masked) for (size_t i = 0; i < pay.size(); i++) pay[i] ^= (char)b[h + (i & 3)];
        c.in.erase(0, h + mh + (size_t)len);
        if (op == 8) { ws_frame(c.out, 8, pay.data(), pay.size() < 2 ? pay.size() : 2); c.closing = true; return; }
        if (op == 9) { ws_frame(c.out, 10, pay.data(), pay.size()); continue; }
        if (op == 10) continue;
        if (op == 1 || op == 2) { c.frag = pay; c.frag_op = op; }
        else if (op == 0 && c.frag_op != 0) c.frag += pay;
        else { c.closing = true; return; }       // a continuation without a start, or a reserved opcode
        if (c.frag.size() > kMaxMessage) { c.closing = true; return; }
        if (fin) {
            if (c.frag_op == 1) {
                if (c.msgs.size() >= kMaxQueued) { c.closing = true; return; }
                c.msgs.push_back(std::move(c.frag));
            }
            c.frag.clear();
            c.frag_op = 0;
        }
    }
}

}  // namespace ppws
