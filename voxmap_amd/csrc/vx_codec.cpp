// vx_codec.cpp — asset containers of the reference (render.js:52-58,
// utils.js:10-30, encrypt.js:1-46, makefile:70-86):
//   .bin     raw bytes
//   .bin.gz  gzip (RFC 1952) of the raw bytes
//   .blob    AES-256-CBC, PKCS#7 padding, fixed IV, of the gzip bytes; the key
//            is a JWK "k" member (base64url of 32 bytes).
#include <openssl/evp.h>
#include <zlib.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "vx_internal.h"

namespace vx {

// utils.js:11-16 == encrypt.js:12-17
static const unsigned char kFixedIV[16] = {55, 44, 146, 89, 30, 93, 68, 30, 209, 23, 56, 140, 88, 149, 55, 221};

static int b64url_val(char c) {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '-' || c == '+') return 62;
    if (c == '_' || c == '/') return 63;
    return -1;
}

// JWK "k" -> 32 raw key bytes (RFC 7518 §6.4.1: base64url, no padding).
int jwk_key(const char *k, unsigned char key[32]) {
    if (!k) return set_error(VX_ECRYPTO, "blob format needs key_jwk_k");
    std::vector<unsigned char> out;
    unsigned acc = 0;
    int bits = 0;
    for (const char *p = k; *p; ++p) {
        if (*p == '=') break;
        int v = b64url_val(*p);
        if (v < 0) return set_error(VX_ECRYPTO, "key_jwk_k is not base64url");
        acc = (acc << 6) | (unsigned)v;
        bits += 6;
        if (bits >= 8) {
            bits -= 8;
            out.push_back((unsigned char)((acc >> bits) & 0xffu));
        }
    }
    if (out.size() != 32) return set_error(VX_ECRYPTO, "key_jwk_k must decode to 32 bytes (A256CBC), got " +
                                                           std::to_string(out.size()));
    std::memcpy(key, out.data(), 32);
    return VX_OK;
}

static int aes_cbc(bool enc, const unsigned char *in, size_t n, const unsigned char key[32],
                   std::vector<unsigned char> &out) {
    EVP_CIPHER_CTX *ctx = EVP_CIPHER_CTX_new();
    if (!ctx) return set_error(VX_ENOMEM, "EVP_CIPHER_CTX_new failed");
    out.resize(n + 32);
    int l1 = 0, l2 = 0;
    int ok = enc ? EVP_EncryptInit_ex(ctx, EVP_aes_256_cbc(), nullptr, key, kFixedIV)
                 : EVP_DecryptInit_ex(ctx, EVP_aes_256_cbc(), nullptr, key, kFixedIV);
    if (ok) ok = enc ? EVP_EncryptUpdate(ctx, out.data(), &l1, in, (int)n) : EVP_DecryptUpdate(ctx, out.data(), &l1, in, (int)n);
    if (ok) ok = enc ? EVP_EncryptFinal_ex(ctx, out.data() + l1, &l2) : EVP_DecryptFinal_ex(ctx, out.data() + l1, &l2);
    EVP_CIPHER_CTX_free(ctx);
    if (!ok) return set_error(VX_ECRYPTO, enc ? "AES-256-CBC encryption failed"
                                              : "AES-256-CBC decryption failed (wrong key or corrupt blob: bad padding)");
    out.resize((size_t)l1 + (size_t)l2);
    return VX_OK;
}

static constexpr size_t kMaxInflate = (size_t)1 << 32;

static int gunzip(const unsigned char *in, size_t n, std::vector<unsigned char> &out, size_t expect) {
    z_stream zs;
    std::memset(&zs, 0, sizeof zs);
    if (inflateInit2(&zs, 15 + 16) != Z_OK) return set_error(VX_EFORMAT, "inflateInit2 failed");
    out.resize(expect ? expect : (n * 4 + 1024));
    zs.next_in = const_cast<unsigned char *>(in);
    zs.avail_in = (uInt)n;
    int rc = Z_OK;
    size_t produced = 0;
    for (;;) {
        if (produced == out.size()) {
            // a known size bounds the output: a stream that inflates past it is
            // rejected without growing further (no unbounded allocation)
            if (expect && produced > expect) {
                inflateEnd(&zs);
                return set_error(VX_ESIZE, "gzip stream inflates past the expected " + std::to_string(expect) + " bytes");
            }
            // an unknown size (vx_decode) is still bounded: no asset of this
            // path is near 4 GiB (the C5 field is 0.9 GB), a gzip bomb is
            if (!expect && produced >= kMaxInflate) {
                inflateEnd(&zs);
                return set_error(VX_ESIZE, "gzip stream inflates past 4 GiB");
            }
            out.resize(expect && produced == expect ? expect + 1 : out.size() * 2 + 1);
        }
        zs.next_out = out.data() + produced;
        zs.avail_out = (uInt)(out.size() - produced);
        rc = inflate(&zs, Z_NO_FLUSH);
        produced = out.size() - zs.avail_out;
        if (rc == Z_STREAM_END) break;
        if (rc != Z_OK && rc != Z_BUF_ERROR) break;
        if (rc == Z_BUF_ERROR && zs.avail_in == 0) break;
    }
    inflateEnd(&zs);
    if (rc != Z_STREAM_END) return set_error(VX_EFORMAT, "gzip stream is corrupt or truncated (zlib rc " + std::to_string(rc) + ")");
    out.resize(produced);
    return VX_OK;
}

int decode_container(const unsigned char *in, size_t n, int format, const char *key,
                     std::vector<unsigned char> &out, size_t expect) {
    if (format == VX_FORMAT_BIN) {
        out.assign(in, in + n);
        return VX_OK;
    }
    // zlib counts input in 32 bits and EVP in a signed int: larger inputs are no asset of this path
    if ((format == VX_FORMAT_BIN_GZ || format == VX_FORMAT_BLOB) && n > (size_t)INT32_MAX)
        return set_error(VX_ESIZE, "container of " + std::to_string(n) + " bytes is too large");
    if (format == VX_FORMAT_BIN_GZ) return gunzip(in, n, out, expect);
    if (format == VX_FORMAT_BLOB) {
        if (n == 0 || n % 16 != 0)
            return set_error(VX_ECRYPTO, "blob size " + std::to_string(n) + " is not a positive multiple of the AES block");
        unsigned char k[32];
        int rc = jwk_key(key, k);
        if (rc) return rc;
        std::vector<unsigned char> gz;
        rc = aes_cbc(false, in, n, k, gz);
        if (rc) return rc;
        return gunzip(gz.data(), gz.size(), out, expect);
    }
    return set_error(VX_EINVAL, "unknown container format " + std::to_string(format));
}

int format_from_path(const char *path) {
    std::string p(path ? path : "");
    auto ends = [&](const char *suf) {
        size_t l = std::strlen(suf);
        return p.size() >= l && p.compare(p.size() - l, l, suf) == 0;
    };
    if (ends(".blob")) return VX_FORMAT_BLOB;
    if (ends(".gz")) return VX_FORMAT_BIN_GZ;
    return VX_FORMAT_BIN;
}

int encrypt_blob(const unsigned char *in, size_t n, const char *key, std::vector<unsigned char> &out) {
    unsigned char k[32];
    int rc = jwk_key(key, k);
    if (rc) return rc;
    return aes_cbc(true, in, n, k, out);
}

}  // namespace vx
