/* sha256.h -- streaming SHA-256 (TEST INFRASTRUCTURE ONLY, see sha256.c). */
#ifndef RFEC_ORACLE_SHA256_H_
#define RFEC_ORACLE_SHA256_H_

#include <stddef.h>
#include <stdint.h>

typedef struct {
    uint32_t h[8];
    uint64_t bytes;
    uint8_t buf[64];
    size_t fill;
} sha256_ctx;

void sha256_init(sha256_ctx* c);
void sha256_update(sha256_ctx* c, const void* data, size_t n);
void sha256_final(sha256_ctx* c, uint8_t out[32]);
void sha256_hex(const uint8_t d[32], char out[65]);

#endif
