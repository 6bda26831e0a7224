/* Fp2 / Fp6 / Fp12 tower (TEST INFRASTRUCTURE: C oracle only).
 *
 * Include-template after field_tmpl.h.  Define before including:
 *   T_(x)   name mangler        FP  base-field type (and FP_(x) its mangler)
 *   XI_A    xi = XI_A + u  (1 for BLS12-381, 9 for BN254)
 * Fp2 = Fp[u]/(u^2+1); Fp6 = Fp2[v]/(v^3 - xi); Fp12 = Fp6[w]/(w^2 - v).
 * Schoolbook formulas (the HIP path uses Karatsuba/Granger-Scott; this restatement is
 * deliberately the plain definition).  Spec: BASELINE.json:5; reference: LICENSE only.
 */
typedef struct { FP c0, c1; } T_(fp2);
typedef struct { T_(fp2) c0, c1, c2; } T_(fp6);
typedef struct { T_(fp6) c0, c1; } T_(fp12);

static inline void T_(fp2_add)(T_(fp2)* r, const T_(fp2)* a, const T_(fp2)* b) {
  FP_(add)(&r->c0, &a->c0, &b->c0); FP_(add)(&r->c1, &a->c1, &b->c1);
}
static inline void T_(fp2_sub)(T_(fp2)* r, const T_(fp2)* a, const T_(fp2)* b) {
  FP_(sub)(&r->c0, &a->c0, &b->c0); FP_(sub)(&r->c1, &a->c1, &b->c1);
}
static inline void T_(fp2_neg)(T_(fp2)* r, const T_(fp2)* a) {
  FP_(neg)(&r->c0, &a->c0); FP_(neg)(&r->c1, &a->c1);
}
static inline void T_(fp2_mul)(T_(fp2)* r, const T_(fp2)* a, const T_(fp2)* b) {
  FP t0, t1, t2, t3;
  FP_(mul)(&t0, &a->c0, &b->c0);
  FP_(mul)(&t1, &a->c1, &b->c1);
  FP_(mul)(&t2, &a->c0, &b->c1);
  FP_(mul)(&t3, &a->c1, &b->c0);
  FP_(sub)(&r->c0, &t0, &t1);
  FP_(add)(&r->c1, &t2, &t3);
}
static inline void T_(fp2_mul_fp)(T_(fp2)* r, const T_(fp2)* a, const FP* s) {
  FP_(mul)(&r->c0, &a->c0, s); FP_(mul)(&r->c1, &a->c1, s);
}
static inline void T_(fp2_conj)(T_(fp2)* r, const T_(fp2)* a) {
  r->c0 = a->c0; FP_(neg)(&r->c1, &a->c1);
}
static inline int T_(fp2_is_zero)(const T_(fp2)* a) { return FP_(is_zero)(&a->c0) && FP_(is_zero)(&a->c1); }
static inline int T_(fp2_eq)(const T_(fp2)* a, const T_(fp2)* b) { return FP_(eq)(&a->c0, &b->c0) && FP_(eq)(&a->c1, &b->c1); }
static inline void T_(fp2_zero)(T_(fp2)* r) { FP_(zero)(&r->c0); FP_(zero)(&r->c1); }
static inline void T_(fp2_one)(T_(fp2)* r) { FP_(one)(&r->c0); FP_(zero)(&r->c1); }
static inline void T_(fp2_small)(T_(fp2)* r, uint64_t a, uint64_t b) {
  uint64_t raw[sizeof(FP) / 8];
  memset(raw, 0, sizeof(raw)); raw[0] = a; FP_(to_mont)(&r->c0, raw);
  memset(raw, 0, sizeof(raw)); raw[0] = b; FP_(to_mont)(&r->c1, raw);
}
static inline void T_(fp2_mul_xi)(T_(fp2)* r, const T_(fp2)* a) {
  T_(fp2) xi; T_(fp2_small)(&xi, XI_A, 1);
  T_(fp2_mul)(r, a, &xi);
}
static inline void T_(fp2_inv)(T_(fp2)* r, const T_(fp2)* a) {
  FP n, t, ni;
  FP_(sqr)(&n, &a->c0); FP_(sqr)(&t, &a->c1); FP_(add)(&n, &n, &t);
  FP_(inv)(&ni, &n);
  FP_(mul)(&r->c0, &a->c0, &ni);
  FP_(mul)(&t, &a->c1, &ni); FP_(neg)(&r->c1, &t);
}
static inline void T_(fp2_pow)(T_(fp2)* r, const T_(fp2)* a, const uint64_t* e, int bits) {
  T_(fp2) acc; T_(fp2_one)(&acc);
  for (int i = bits - 1; i >= 0; --i) {
    T_(fp2_mul)(&acc, &acc, &acc);
    if ((e[i / 64] >> (i % 64)) & 1) T_(fp2_mul)(&acc, &acc, a);
  }
  *r = acc;
}

static inline void T_(fp6_add)(T_(fp6)* r, const T_(fp6)* a, const T_(fp6)* b) {
  T_(fp2_add)(&r->c0, &a->c0, &b->c0); T_(fp2_add)(&r->c1, &a->c1, &b->c1); T_(fp2_add)(&r->c2, &a->c2, &b->c2);
}
static inline void T_(fp6_neg)(T_(fp6)* r, const T_(fp6)* a) {
  T_(fp2_neg)(&r->c0, &a->c0); T_(fp2_neg)(&r->c1, &a->c1); T_(fp2_neg)(&r->c2, &a->c2);
}
/* schoolbook: c0 = a0b0 + xi(a1b2 + a2b1); c1 = a0b1 + a1b0 + xi a2b2; c2 = a0b2 + a1b1 + a2b0 */
static inline void T_(fp6_mul)(T_(fp6)* r, const T_(fp6)* a, const T_(fp6)* b) {
  T_(fp2) t, u, c0, c1, c2;
  T_(fp2_mul)(&c0, &a->c0, &b->c0);
  T_(fp2_mul)(&t, &a->c1, &b->c2); T_(fp2_mul)(&u, &a->c2, &b->c1); T_(fp2_add)(&t, &t, &u);
  T_(fp2_mul_xi)(&t, &t); T_(fp2_add)(&c0, &c0, &t);
  T_(fp2_mul)(&c1, &a->c0, &b->c1);
  T_(fp2_mul)(&t, &a->c1, &b->c0); T_(fp2_add)(&c1, &c1, &t);
  T_(fp2_mul)(&t, &a->c2, &b->c2); T_(fp2_mul_xi)(&t, &t); T_(fp2_add)(&c1, &c1, &t);
  T_(fp2_mul)(&c2, &a->c0, &b->c2);
  T_(fp2_mul)(&t, &a->c1, &b->c1); T_(fp2_add)(&c2, &c2, &t);
  T_(fp2_mul)(&t, &a->c2, &b->c0); T_(fp2_add)(&c2, &c2, &t);
  r->c0 = c0; r->c1 = c1; r->c2 = c2;
}
/* multiply by v: (x0, x1, x2) -> (xi x2, x0, x1) */
static inline void T_(fp6_mul_v)(T_(fp6)* r, const T_(fp6)* a) {
  T_(fp2) t; T_(fp2_mul_xi)(&t, &a->c2);
  T_(fp2) a0 = a->c0, a1 = a->c1;
  r->c0 = t; r->c1 = a0; r->c2 = a1;
}

static inline void T_(fp12_one)(T_(fp12)* r) {
  memset(r, 0, sizeof(*r)); T_(fp2_one)(&r->c0.c0);
}
static inline void T_(fp12_mul)(T_(fp12)* r, const T_(fp12)* a, const T_(fp12)* b) {
  T_(fp6) t0, t1, t2, t3;
  T_(fp6_mul)(&t0, &a->c0, &b->c0);
  T_(fp6_mul)(&t1, &a->c1, &b->c1);
  T_(fp6_mul_v)(&t1, &t1);
  T_(fp6_mul)(&t2, &a->c0, &b->c1);
  T_(fp6_mul)(&t3, &a->c1, &b->c0);
  T_(fp6_add)(&r->c0, &t0, &t1);
  T_(fp6_add)(&r->c1, &t2, &t3);
}
static inline void T_(fp12_conj)(T_(fp12)* r, const T_(fp12)* a) {
  r->c0 = a->c0; T_(fp6_neg)(&r->c1, &a->c1);
}
static inline int T_(fp12_is_one)(const T_(fp12)* a) {
  T_(fp12) one; T_(fp12_one)(&one);
  return memcmp(a, &one, sizeof(one)) == 0;
}
static inline void T_(fp12_pow)(T_(fp12)* r, const T_(fp12)* a, const uint64_t* e, int bits) {
  T_(fp12) acc; T_(fp12_one)(&acc);
  for (int i = bits - 1; i >= 0; --i) {
    T_(fp12_mul)(&acc, &acc, &acc);
    if ((e[i / 64] >> (i % 64)) & 1) T_(fp12_mul)(&acc, &acc, a);
  }
  *r = acc;
}
