// oryx_keystore.cpp -- the HTTPS front end's Java keystores.
//
// The reference hands oryx.serving.api.keystore-file / keystore-password to Tomcat's connector
// as a Java keystore ([lserving]/ServingLayer.java:214-217; its IT serves HTTPS from a JKS file,
// SecureAPIConfigIT.java:84-86).  Here the same two keys accept:
//
//   * JKS (magic 0xFEEDFEED, versions 1 and 2): the file digest is checked -- SHA-1 over the
//     password as UTF-16BE, the bytes "Mighty Aphrodite" and the file body -- and the first
//     private-key entry (or the named alias) is decrypted with the JDK key protector
//     (OID 1.3.6.1.4.1.42.2.17.1.1: salt(20) || ciphertext || check(20); the key stream is
//     SHA-1(password || salt), then SHA-1(password || previous block); the check is
//     SHA-1(password || plaintext)); the plaintext is a PKCS#8 PrivateKeyInfo.  Certificates are
//     DER X.509, leaf first.
//   * PKCS#12 (keytool's default since JDK 9, `openssl pkcs12 -export`): OpenSSL's parser, with
//     the legacy provider loaded when present (RC2 / 3DES-protected files from older JDKs).
//   * anything else -- PEM -- is left to the caller (kKeystoreNotKeystore).
//
// Nothing here executes content from the file: it is parsed as data only.  The password is
// used as the key password too, as Tomcat does when keyPass is not set.
#include "oryx_keystore.h"

#include <openssl/bio.h>
#include <openssl/err.h>
#include <openssl/objects.h>
#include <openssl/pem.h>
#include <openssl/pkcs12.h>
#include <openssl/provider.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

namespace oryx {
namespace {

bool read_file(const char* path, std::vector<unsigned char>* out) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  unsigned char buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof(buf), f)) > 0) out->insert(out->end(), buf, buf + n);
  const bool ok = !ferror(f);
  fclose(f);
  return ok;
}

// UTF-8 -> the UTF-16BE bytes of Java's char[] password (surrogate pairs above the BMP)
std::vector<unsigned char> java_password(const char* pw) {
  std::vector<unsigned char> out;
  const unsigned char* s = reinterpret_cast<const unsigned char*>(pw ? pw : "");
  auto put = [&](unsigned u) {
    out.push_back((unsigned char)(u >> 8));
    out.push_back((unsigned char)(u & 0xFF));
  };
  while (*s) {
    unsigned cp;
    int extra;
    if (*s < 0x80) {
      cp = *s;
      extra = 0;
    } else if ((*s & 0xE0) == 0xC0) {
      cp = *s & 0x1F;
      extra = 1;
    } else if ((*s & 0xF0) == 0xE0) {
      cp = *s & 0x0F;
      extra = 2;
    } else {
      cp = *s & 0x07;
      extra = 3;
    }
    ++s;
    for (int i = 0; i < extra && (*s & 0xC0) == 0x80; ++i, ++s) cp = (cp << 6) | (*s & 0x3F);
    if (cp >= 0x10000) {
      cp -= 0x10000;
      put(0xD800 + (cp >> 10));
      put(0xDC00 + (cp & 0x3FF));
    } else {
      put(cp);
    }
  }
  return out;
}

struct Reader {
  const unsigned char* p;
  const unsigned char* end;
  bool ok = true;
  bool need(size_t n) {
    if (!ok || (size_t)(end - p) < n) ok = false;
    return ok;
  }
  uint32_t u32() {
    if (!need(4)) return 0;
    const uint32_t v = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
    p += 4;
    return v;
  }
  uint16_t u16() {
    if (!need(2)) return 0;
    const uint16_t v = (uint16_t)((p[0] << 8) | p[1]);
    p += 2;
    return v;
  }
  std::string utf() {   // Java DataOutput.writeUTF: u16 length + modified UTF-8
    const uint16_t n = u16();
    if (!need(n)) return std::string();
    std::string s(reinterpret_cast<const char*>(p), n);
    p += n;
    return s;
  }
  const unsigned char* bytes(size_t n) {
    if (!need(n)) return nullptr;
    const unsigned char* q = p;
    p += n;
    return q;
  }
};

void sha1_parts(const std::vector<unsigned char>& a, const unsigned char* b, size_t nb,
                const unsigned char* c, size_t nc, unsigned char out[20]) {
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  EVP_DigestInit_ex(ctx, EVP_sha1(), nullptr);
  EVP_DigestUpdate(ctx, a.data(), a.size());
  if (nb) EVP_DigestUpdate(ctx, b, nb);
  if (nc) EVP_DigestUpdate(ctx, c, nc);
  unsigned int n = 20;
  EVP_DigestFinal_ex(ctx, out, &n);
  EVP_MD_CTX_free(ctx);
}

bool iequal(const std::string& a, const char* b) {
  if (a.size() != strlen(b)) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (tolower((unsigned char)a[i]) != tolower((unsigned char)b[i])) return false;
  return true;
}

std::string ssl_error(const char* what) {
  char eb[256];
  const unsigned long e = ERR_get_error();
  ERR_error_string_n(e, eb, sizeof(eb));
  ERR_clear_error();
  return std::string(what) + (e ? std::string(": ") + eb : std::string());
}

// JDK key protector (sun.security.provider.KeyProtector.recover) -> PKCS#8 DER
int jks_recover_key(const unsigned char* der, size_t n, const std::vector<unsigned char>& pw,
                    std::vector<unsigned char>* plain, std::string* err) {
  const unsigned char* q = der;
  X509_SIG* epki = d2i_X509_SIG(nullptr, &q, (long)n);
  if (!epki) {
    *err = "JKS key entry is not an EncryptedPrivateKeyInfo";
    return kKeystoreMalformed;
  }
  const X509_ALGOR* alg = nullptr;
  const ASN1_OCTET_STRING* data = nullptr;
  X509_SIG_get0(epki, &alg, &data);
  char oid[80];
  OBJ_obj2txt(oid, sizeof(oid), alg->algorithm, 1);
  if (strcmp(oid, "1.3.6.1.4.1.42.2.17.1.1") != 0) {
    X509_SIG_free(epki);
    *err = std::string("JKS key protection ") + oid + " is not supported";
    return kKeystoreUnsupported;
  }
  const unsigned char* d = ASN1_STRING_get0_data(data);
  const size_t dn = (size_t)ASN1_STRING_length(data);
  if (dn < 40) {
    X509_SIG_free(epki);
    *err = "JKS protected key too short";
    return kKeystoreMalformed;
  }
  const unsigned char* salt = d;
  const unsigned char* enc = d + 20;
  const size_t en = dn - 40;
  const unsigned char* check = d + dn - 20;
  plain->resize(en);
  unsigned char block[20];
  memcpy(block, salt, 20);
  for (size_t off = 0; off < en; off += 20) {
    unsigned char next[20];
    sha1_parts(pw, block, 20, nullptr, 0, next);
    memcpy(block, next, 20);
    const size_t m = en - off < 20 ? en - off : 20;
    for (size_t i = 0; i < m; ++i) (*plain)[off + i] = enc[off + i] ^ block[i];
  }
  unsigned char got[20];
  sha1_parts(pw, plain->data(), plain->size(), nullptr, 0, got);
  // (check points into epki's octet string: compared before epki is freed)
  const bool match = memcmp(got, check, 20) == 0;
  X509_SIG_free(epki);
  if (!match) {
    *err = "JKS private key: wrong password";
    return kKeystoreBadPassword;
  }
  return kKeystoreOk;
}

int load_jks(const std::vector<unsigned char>& f, const char* password, const char* alias,
             EVP_PKEY** key, X509** cert, STACK_OF(X509)** chain, std::string* err) {
  if (f.size() < 12 + 20) {
    *err = "JKS file truncated";
    return kKeystoreMalformed;
  }
  const std::vector<unsigned char> pw = java_password(password);
  if (password) {
    static const char kWhitener[] = "Mighty Aphrodite";
    unsigned char dig[20];
    sha1_parts(pw, reinterpret_cast<const unsigned char*>(kWhitener), strlen(kWhitener),
               f.data(), f.size() - 20, dig);
    if (memcmp(dig, f.data() + f.size() - 20, 20) != 0) {
      *err = "JKS keystore integrity check failed: wrong password or a corrupt file";
      return kKeystoreBadPassword;
    }
  }
  Reader r{f.data() + 4, f.data() + f.size() - 20};
  const uint32_t version = r.u32();
  if (version != 1 && version != 2) {
    *err = "JKS version " + std::to_string(version) + " is not supported";
    return kKeystoreUnsupported;
  }
  const uint32_t count = r.u32();
  for (uint32_t e = 0; e < count && r.ok; ++e) {
    const uint32_t tag = r.u32();
    const std::string name = r.utf();
    r.bytes(8);   // creation time
    if (tag == 2) {   // trusted certificate entry
      if (version == 2) r.utf();
      const uint32_t n = r.u32();
      r.bytes(n);
      continue;
    }
    if (tag != 1) {
      *err = "JKS entry tag " + std::to_string(tag) + " is not supported";
      return kKeystoreMalformed;
    }
    const uint32_t kn = r.u32();
    const unsigned char* kd = r.bytes(kn);
    const uint32_t nc = r.u32();
    std::vector<std::pair<const unsigned char*, uint32_t>> certs;
    for (uint32_t c = 0; c < nc && r.ok; ++c) {
      if (version == 2) r.utf();
      const uint32_t cn = r.u32();
      const unsigned char* cd = r.bytes(cn);
      certs.emplace_back(cd, cn);
    }
    if (!r.ok) break;
    if (alias && *alias && !iequal(name, alias)) continue;
    std::vector<unsigned char> plain;
    const int rc = jks_recover_key(kd, kn, pw, &plain, err);
    if (rc != kKeystoreOk) return rc;
    const unsigned char* q = plain.data();
    PKCS8_PRIV_KEY_INFO* p8 = d2i_PKCS8_PRIV_KEY_INFO(nullptr, &q, (long)plain.size());
    OPENSSL_cleanse(plain.data(), plain.size());
    if (!p8) {
      *err = ssl_error("JKS private key is not PKCS#8");
      return kKeystoreMalformed;
    }
    EVP_PKEY* k = EVP_PKCS82PKEY(p8);
    PKCS8_PRIV_KEY_INFO_free(p8);
    if (!k) {
      *err = ssl_error("JKS private key");
      return kKeystoreMalformed;
    }
    if (certs.empty()) {
      EVP_PKEY_free(k);
      *err = "JKS key entry has no certificate";
      return kKeystoreMalformed;
    }
    STACK_OF(X509)* st = sk_X509_new_null();
    X509* leaf = nullptr;
    for (size_t c = 0; c < certs.size(); ++c) {
      const unsigned char* cq = certs[c].first;
      X509* x = d2i_X509(nullptr, &cq, (long)certs[c].second);
      if (!x) {
        EVP_PKEY_free(k);
        X509_free(leaf);
        sk_X509_pop_free(st, X509_free);
        *err = ssl_error("JKS certificate");
        return kKeystoreMalformed;
      }
      if (c == 0) leaf = x;
      else sk_X509_push(st, x);
    }
    *key = k;
    *cert = leaf;
    *chain = st;
    return kKeystoreOk;
  }
  if (!r.ok) {
    *err = "JKS file truncated";
    return kKeystoreMalformed;
  }
  *err = alias && *alias ? std::string("JKS keystore has no private-key entry '") + alias + "'"
                         : std::string("JKS keystore has no private-key entry");
  return kKeystoreUnsupported;
}

void load_legacy_provider() {
  static std::once_flag once;
  std::call_once(once, [] {
    // loading any provider into the default context turns off its implicit default
    // provider: load both (legacy is absent on some systems -- then only modern PBE works)
    if (OSSL_PROVIDER_load(nullptr, "legacy")) OSSL_PROVIDER_load(nullptr, "default");
    ERR_clear_error();
  });
}

int load_p12(const std::vector<unsigned char>& f, const char* password, EVP_PKEY** key,
             X509** cert, STACK_OF(X509)** chain, std::string* err) {
  load_legacy_provider();
  const unsigned char* q = f.data();
  PKCS12* p12 = d2i_PKCS12(nullptr, &q, (long)f.size());
  if (!p12) {
    ERR_clear_error();
    return kKeystoreNotKeystore;
  }
  const char* pw = password ? password : "";
  if (PKCS12_mac_present(p12) && !PKCS12_verify_mac(p12, pw, -1)) {
    PKCS12_free(p12);
    *err = ssl_error("PKCS#12 keystore: wrong password (MAC check failed)");
    return kKeystoreBadPassword;
  }
  EVP_PKEY* k = nullptr;
  X509* x = nullptr;
  STACK_OF(X509)* ca = nullptr;
  const int ok = PKCS12_parse(p12, pw, &k, &x, &ca);
  PKCS12_free(p12);
  if (!ok) {
    *err = ssl_error("PKCS#12 keystore");
    return kKeystoreMalformed;
  }
  if (!k || !x) {
    EVP_PKEY_free(k);
    X509_free(x);
    sk_X509_pop_free(ca, X509_free);
    *err = "PKCS#12 keystore has no private key with a certificate";
    return kKeystoreUnsupported;
  }
  *key = k;
  *cert = x;
  *chain = ca ? ca : sk_X509_new_null();
  return kKeystoreOk;
}

}  // namespace

int keystore_load(const char* path, const char* password, const char* alias, EVP_PKEY** key,
                  X509** cert, STACK_OF(X509)** chain, std::string* err) {
  std::vector<unsigned char> f;
  if (!read_file(path, &f)) {
    *err = std::string("cannot read keystore ") + path;
    return kKeystoreIO;
  }
  if (f.size() >= 4 && f[0] == 0xFE && f[1] == 0xED && f[2] == 0xFE && f[3] == 0xED)
    return load_jks(f, password, alias, key, cert, chain, err);
  if (f.size() >= 4 && f[0] == 0xCE && f[1] == 0xCE && f[2] == 0xCE && f[3] == 0xCE) {
    *err = "JCEKS keystores are not supported (convert with keytool -importkeystore to PKCS12)";
    return kKeystoreUnsupported;
  }
  if (!f.empty() && f[0] == 0x30) return load_p12(f, password, key, cert, chain, err);
  return kKeystoreNotKeystore;
}

}  // namespace oryx

namespace {
thread_local std::string ks_err;

char* bio_string(BIO* b, long long* len) {
  char* data = nullptr;
  const long n = BIO_get_mem_data(b, &data);
  char* out = static_cast<char*>(malloc((size_t)n + 1));
  if (!out) return nullptr;
  memcpy(out, data, (size_t)n);
  out[n] = 0;
  *len = n;
  return out;
}
}  // namespace

extern "C" {

// The keystore at `path` as PEM text: the certificate chain (leaf first) and the unencrypted
// PKCS#8 private key, malloc'ed (oryx_keystore_free).  Returns an oryx::KeystoreStatus;
// oryx_keystore_error() says why on failure.  (For the Python-side TLS context; the native
// front end loads keystores without going through PEM.)
int oryx_keystore_to_pem(const char* path, const char* password, const char* alias,
                         char** cert_pem, long long* cert_len, char** key_pem,
                         long long* key_len) {
  ks_err.clear();
  EVP_PKEY* key = nullptr;
  X509* cert = nullptr;
  STACK_OF(X509)* chain = nullptr;
  const int rc = oryx::keystore_load(path, password, alias, &key, &cert, &chain, &ks_err);
  if (rc != oryx::kKeystoreOk) return rc;
  BIO* cb = BIO_new(BIO_s_mem());
  BIO* kb = BIO_new(BIO_s_mem());
  bool ok = cb && kb && PEM_write_bio_X509(cb, cert) == 1;
  for (int i = 0; ok && i < sk_X509_num(chain); ++i)
    ok = PEM_write_bio_X509(cb, sk_X509_value(chain, i)) == 1;
  ok = ok && PEM_write_bio_PrivateKey(kb, key, nullptr, nullptr, 0, nullptr, nullptr) == 1;
  if (ok) {
    *cert_pem = bio_string(cb, cert_len);
    *key_pem = bio_string(kb, key_len);
    ok = *cert_pem && *key_pem;
  }
  if (!ok) ks_err = "PEM encoding failed";
  BIO_free(cb);
  BIO_free(kb);
  EVP_PKEY_free(key);
  X509_free(cert);
  sk_X509_pop_free(chain, X509_free);
  return ok ? oryx::kKeystoreOk : oryx::kKeystoreMalformed;
}

void oryx_keystore_free(char* p) {
  if (p) {
    OPENSSL_cleanse(p, strlen(p));
    free(p);
  }
}

const char* oryx_keystore_error() { return ks_err.c_str(); }

}  // extern "C"
