/* Montgomery prime field over 64-bit limbs (TEST INFRASTRUCTURE: C oracle only).
 *
 * Include-template: before including define
 *   F      type name          FN     limb count (64-bit)
 *   F_(x)  name mangler       FMOD / FRR / FR2 / FINV   constants from consts_gen.h
 * Restates the standard CIOS Montgomery multiplication with unsigned __int128 (independent
 * of the HIP kernels, which use 32-bit limbs and v_mad_u64_u32).  Spec: BASELINE.json:5;
 * reference: none (/root/reference/LICENSE:1-201 only).
 */
typedef struct { uint64_t v[FN]; } F;

static inline void F_(zero)(F* r) { memset(r, 0, sizeof(F)); }
static inline void F_(one)(F* r) { memcpy(r->v, FRR, sizeof(F)); }
static inline int F_(is_zero)(const F* a) {
  uint64_t x = 0;
  for (int i = 0; i < FN; ++i) x |= a->v[i];
  return x == 0;
}
static inline int F_(eq)(const F* a, const F* b) { return memcmp(a, b, sizeof(F)) == 0; }
static inline int F_(is_one)(const F* a) { return memcmp(a->v, FRR, sizeof(F)) == 0; }

/* a >= MOD ? (raw comparison of FN limbs) */
static inline int F_(geq_mod)(const uint64_t* a) {
  for (int i = FN - 1; i >= 0; --i) {
    if (a[i] > FMOD[i]) return 1;
    if (a[i] < FMOD[i]) return 0;
  }
  return 1;
}

static inline void F_(add)(F* r, const F* a, const F* b) {
  uint64_t t[FN];
  unsigned __int128 c = 0;
  for (int i = 0; i < FN; ++i) { c += (unsigned __int128)a->v[i] + b->v[i]; t[i] = (uint64_t)c; c >>= 64; }
  if (c || F_(geq_mod)(t)) {
    unsigned __int128 bw = 0;
    for (int i = 0; i < FN; ++i) {
      unsigned __int128 d = (unsigned __int128)t[i] - FMOD[i] - (uint64_t)bw;
      t[i] = (uint64_t)d; bw = (d >> 64) ? 1 : 0;
    }
  }
  memcpy(r->v, t, sizeof(t));
}

static inline void F_(sub)(F* r, const F* a, const F* b) {
  uint64_t t[FN];
  unsigned __int128 bw = 0;
  for (int i = 0; i < FN; ++i) {
    unsigned __int128 d = (unsigned __int128)a->v[i] - b->v[i] - (uint64_t)bw;
    t[i] = (uint64_t)d; bw = (d >> 64) ? 1 : 0;
  }
  if (bw) {
    unsigned __int128 c = 0;
    for (int i = 0; i < FN; ++i) { c += (unsigned __int128)t[i] + FMOD[i]; t[i] = (uint64_t)c; c >>= 64; }
  }
  memcpy(r->v, t, sizeof(t));
}

static inline void F_(neg)(F* r, const F* a) {
  F z; F_(zero)(&z); F_(sub)(r, &z, a);
}

static inline void F_(dbl)(F* r, const F* a) { F_(add)(r, a, a); }

static inline void F_(mul)(F* r, const F* a, const F* b) {
  uint64_t t[FN + 2];
  memset(t, 0, sizeof(t));
  for (int i = 0; i < FN; ++i) {
    unsigned __int128 c = 0;
    for (int j = 0; j < FN; ++j) {
      c += (unsigned __int128)a->v[j] * b->v[i] + t[j];
      t[j] = (uint64_t)c; c >>= 64;
    }
    c += t[FN]; t[FN] = (uint64_t)c; t[FN + 1] = (uint64_t)(c >> 64);
    uint64_t m = t[0] * FINV;
    c = (unsigned __int128)m * FMOD[0] + t[0];
    c >>= 64;
    for (int j = 1; j < FN; ++j) {
      c += (unsigned __int128)m * FMOD[j] + t[j];
      t[j - 1] = (uint64_t)c; c >>= 64;
    }
    c += t[FN]; t[FN - 1] = (uint64_t)c; c >>= 64;
    t[FN] = t[FN + 1] + (uint64_t)c;
  }
  if (t[FN] || F_(geq_mod)(t)) {
    unsigned __int128 bw = 0;
    for (int i = 0; i < FN; ++i) {
      unsigned __int128 d = (unsigned __int128)t[i] - FMOD[i] - (uint64_t)bw;
      t[i] = (uint64_t)d; bw = (d >> 64) ? 1 : 0;
    }
  }
  memcpy(r->v, t, sizeof(F));
}

static inline void F_(sqr)(F* r, const F* a) { F_(mul)(r, a, a); }

/* raw (non-Montgomery) integer -> Montgomery form */
static inline void F_(to_mont)(F* r, const uint64_t* raw) {
  F a; memcpy(a.v, raw, sizeof(F));
  F r2; memcpy(r2.v, FR2, sizeof(F));
  F_(mul)(r, &a, &r2);
}
static inline void F_(from_mont)(uint64_t* raw, const F* a) {
  F one; F_(zero)(&one); one.v[0] = 1;
  F t; F_(mul)(&t, a, &one);
  memcpy(raw, t.v, sizeof(F));
}

/* a^e for e given as little-endian 64-bit words with `bits` significant bits */
static inline void F_(pow)(F* r, const F* a, const uint64_t* e, int bits) {
  F acc; F_(one)(&acc);
  for (int i = bits - 1; i >= 0; --i) {
    F_(sqr)(&acc, &acc);
    if ((e[i / 64] >> (i % 64)) & 1) F_(mul)(&acc, &acc, a);
  }
  *r = acc;
}

static inline void F_(inv)(F* r, const F* a) {  /* Fermat: a^(m-2) */
  uint64_t e[FN];
  memcpy(e, FMOD, sizeof(e));
  e[0] -= 2; /* MOD is odd and > 2: no borrow */
  F_(pow)(r, a, e, FN * 64);
}

/* big-endian bytes (FN*8 - pad .. ) -> raw limbs; nbytes <= FN*8 */
static inline void F_(raw_from_be)(uint64_t* raw, const uint8_t* b, int nbytes) {
  memset(raw, 0, FN * 8);
  for (int i = 0; i < nbytes; ++i) {
    int k = nbytes - 1 - i; /* byte significance */
    raw[k / 8] |= (uint64_t)b[i] << (8 * (k % 8));
  }
}
static inline void F_(raw_to_be)(uint8_t* b, const uint64_t* raw, int nbytes) {
  for (int i = 0; i < nbytes; ++i) {
    int k = nbytes - 1 - i;
    b[i] = (uint8_t)(raw[k / 8] >> (8 * (k % 8)));
  }
}
/* canonical decode: returns 0 on success, -1 if value >= MOD */
static inline int F_(from_be)(F* r, const uint8_t* b, int nbytes) {
  uint64_t raw[FN];
  F_(raw_from_be)(raw, b, nbytes);
  if (F_(geq_mod)(raw)) return -1;
  F_(to_mont)(r, raw);
  return 0;
}
static inline void F_(to_be)(uint8_t* b, const F* a, int nbytes) {
  uint64_t raw[FN];
  F_(from_mont)(raw, a);
  F_(raw_to_be)(b, raw, nbytes);
}
