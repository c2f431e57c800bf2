// Java keystores (JKS, PKCS#12) for the HTTPS front end; see oryx_keystore.cpp.
#pragma once

#include <openssl/evp.h>
#include <openssl/x509.h>

#include <string>

namespace oryx {

enum KeystoreStatus {
  kKeystoreOk = 0,
  kKeystoreNotKeystore = 1,   // PEM (or anything else): the caller loads the file as PEM
  kKeystoreBadPassword = 2,   // integrity / MAC / key-protector check failed
  kKeystoreMalformed = 3,
  kKeystoreUnsupported = 4,   // e.g. JCEKS, or no private-key entry
  kKeystoreIO = 5,
};

// The first private-key entry of the keystore at `path` (or the one named `alias` when
// non-empty) with its certificate chain, leaf first.  On kKeystoreOk the caller owns *key,
// *cert and *chain (chain may be empty, never null).
int keystore_load(const char* path, const char* password, const char* alias, EVP_PKEY** key,
                  X509** cert, STACK_OF(X509)** chain, std::string* err);

}  // namespace oryx
