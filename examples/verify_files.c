/* A plain-C caller of the drop-in boundary (include/kzgmi.h), the way a C / Go / Rust host
 * would bind it: load an SRS, verify one batch from host buffers (the PCIe-inclusive entry
 * point), print the verdict and the two combined points A, B.
 *
 *   verify_files CURVE N G2 TAU_G2 COMMITMENTS ZS YS PROOFS SEED
 *
 * CURVE is bls12_381 or bn254; the other arguments are files holding the raw encodings
 * (G2 / [tau]_2 192 or 128 B, N G1 points of 96 or 64 B, N scalars of 32 B, a 32-B seed).
 * Output: "ok=<0|1> A=<hex> B=<hex>"; exit status 0, or the library's error code on stderr
 * with exit status 2 (no GPU: KZGMI_ERR_DEVICE -- there is no CPU fallback).
 * Build: gcc -O2 -I include examples/verify_files.c -L<dir of libkzgmi.so> -lkzgmi
 * (tests/test_c_example.py builds and runs it). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "kzgmi.h"

static unsigned char* slurp(const char* path, size_t want) {
  FILE* f = fopen(path, "rb");
  if (!f) { perror(path); exit(3); }
  unsigned char* buf = malloc(want ? want : 1);
  size_t got = fread(buf, 1, want, f);
  fclose(f);
  if (got != want) { fprintf(stderr, "%s: %zu of %zu bytes\n", path, got, want); exit(3); }
  return buf;
}

static void hex(const char* tag, const unsigned char* p, size_t len) {
  printf(" %s=", tag);
  for (size_t i = 0; i < len; ++i) printf("%02x", p[i]);
}

int main(int argc, char** argv) {
  if (argc != 10) {
    fprintf(stderr, "usage: %s CURVE N G2 TAU_G2 COMMITMENTS ZS YS PROOFS SEED\n", argv[0]);
    return 3;
  }
  const int bls = strcmp(argv[1], "bls12_381") == 0;
  const kzgmi_curve curve = bls ? KZGMI_BLS12_381 : KZGMI_BN254;
  const size_t n = strtoull(argv[2], NULL, 10);
  const size_t g1b = bls ? 96 : 64, g2b = bls ? 192 : 128;
  unsigned char* g2 = slurp(argv[3], g2b);
  unsigned char* tg2 = slurp(argv[4], g2b);
  unsigned char* cm = slurp(argv[5], n * g1b);
  unsigned char* zs = slurp(argv[6], n * 32);
  unsigned char* ys = slurp(argv[7], n * 32);
  unsigned char* pf = slurp(argv[8], n * g1b);
  unsigned char* seed = slurp(argv[9], 32);

  /* a library built for another ABI revision must not be bound (include/kzgmi.h) */
  if (kzgmi_abi_version() != KZGMI_ABI_VERSION) {
    fprintf(stderr, "libkzgmi ABI %d, this program was built for %d\n", kzgmi_abi_version(), KZGMI_ABI_VERSION);
    return 2;
  }
  kzgmi_ctx* ctx = NULL;
  kzgmi_srs* srs = NULL;
  int ok = -1;
  const int devices[1] = {0};
  int rc = kzgmi_ctx_create(&ctx, devices, 1, 1);
  if (!rc) rc = kzgmi_srs_load(ctx, curve, NULL, g2, tg2, &srs);
  if (!rc) rc = kzgmi_batch_verify(ctx, srs, cm, zs, ys, pf, n, seed, &ok);
  unsigned char a[96], b[96];
  if (!rc) rc = kzgmi_last_combination(ctx, a, b);
  if (rc) {
    fprintf(stderr, "kzgmi error %d: %s\n", rc, kzgmi_last_error());
    if (srs) kzgmi_srs_free(srs);
    if (ctx) kzgmi_ctx_destroy(ctx);
    return 2;
  }
  printf("ok=%d", ok);
  hex("A", a, g1b);
  hex("B", b, g1b);
  printf("\n");
  kzgmi_srs_free(srs);
  kzgmi_ctx_destroy(ctx);
  free(g2); free(tg2); free(cm); free(zs); free(ys); free(pf); free(seed);
  return 0;
}
