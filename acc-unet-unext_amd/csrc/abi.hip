// ABI identity of this build: a hash of include/accunet.h taken when this file was
// compiled (the Makefile passes it as ACCUNET_ABI_HASH). accunet/_lib.py hashes the
// header it binds against and refuses a library whose hash differs, so a library
// built from other entry-point signatures is never called with shifted arguments.
#include "common.h"

#ifndef ACCUNET_ABI_HASH
#error "ACCUNET_ABI_HASH must be defined by the build (Makefile)"
#endif

extern "C" long long accunet_abi_hash() { return (long long)ACCUNET_ABI_HASH; }
