/* G1 / G2 / pairing / Pippenger / batch verify for one curve (TEST INFRASTRUCTURE: oracle).
 *
 * Include-template after field_tmpl.h (twice: Fp and Fr) and tower_tmpl.h.  Define:
 *   C_(x) mangler; FP/FP_ base field; FR/FR_ scalar field; T_ tower mangler
 *   FPB  bytes per Fp (48 / 32);  IS_BLS  (ZCash flag encodings, M-type twist, x < 0)
 *   B_SMALL  curve b;  G1X/G1Y raw generator;  FEXP/FEXP_BITS final exponent;
 *   LOOP_WORDS/LOOP_BITS  ate loop integer;  FROB_* and B2_* twist constants.
 *
 * Everything here restates the definitions in oracle/pyspec (itself restating
 * BASELINE.json:5 and SURVEY.md 3.1/8a) with textbook algorithms: Jacobian G1, affine
 * twist Miller loop with full Fp12 line multiplication, naive final exponentiation,
 * unsigned-window Pippenger.  Reference: none (/root/reference/LICENSE:1-201 only).
 */
typedef struct { FP x, y; int inf; } C_(aff);
typedef struct { FP x, y, z; } C_(jac);           /* x = X/Z^2, y = Y/Z^3; Z = 0 <=> O */
typedef struct { T_(fp2) x, y; int inf; } C_(aff2);

/* ------------------------------------------------------------------ G1 Jacobian */
static inline void C_(jac_set_inf)(C_(jac)* r) { FP_(one)(&r->x); FP_(one)(&r->y); FP_(zero)(&r->z); }
static inline int C_(jac_is_inf)(const C_(jac)* a) { return FP_(is_zero)(&a->z); }

static void C_(jac_dbl)(C_(jac)* r, const C_(jac)* p) {
  if (C_(jac_is_inf)(p) || FP_(is_zero)(&p->y)) { C_(jac_set_inf)(r); return; }
  FP A, B, Cc, D, E, Fq, t, X3, Y3, Z3;
  FP_(sqr)(&A, &p->x); FP_(sqr)(&B, &p->y); FP_(sqr)(&Cc, &B);
  FP_(add)(&t, &p->x, &B); FP_(sqr)(&t, &t); FP_(sub)(&t, &t, &A); FP_(sub)(&t, &t, &Cc); FP_(dbl)(&D, &t);
  FP_(dbl)(&E, &A); FP_(add)(&E, &E, &A);
  FP_(sqr)(&Fq, &E);
  FP_(dbl)(&t, &D); FP_(sub)(&X3, &Fq, &t);
  FP_(sub)(&t, &D, &X3); FP_(mul)(&Y3, &E, &t);
  FP_(dbl)(&t, &Cc); FP_(dbl)(&t, &t); FP_(dbl)(&t, &t); FP_(sub)(&Y3, &Y3, &t);
  FP_(mul)(&Z3, &p->y, &p->z); FP_(dbl)(&Z3, &Z3);
  r->x = X3; r->y = Y3; r->z = Z3;
}

static void C_(jac_add_aff)(C_(jac)* r, const C_(jac)* p, const C_(aff)* q) {
  if (q->inf) { *r = *p; return; }
  if (C_(jac_is_inf)(p)) { r->x = q->x; r->y = q->y; FP_(one)(&r->z); return; }
  FP Z1Z1, U2, S2, H, HH, I, J, rr, V, t, X3, Y3, Z3;
  FP_(sqr)(&Z1Z1, &p->z);
  FP_(mul)(&U2, &q->x, &Z1Z1);
  FP_(mul)(&S2, &q->y, &p->z); FP_(mul)(&S2, &S2, &Z1Z1);
  FP_(sub)(&H, &U2, &p->x);
  FP_(sub)(&rr, &S2, &p->y);
  if (FP_(is_zero)(&H)) {
    if (FP_(is_zero)(&rr)) { C_(jac_dbl)(r, p); return; }
    C_(jac_set_inf)(r); return;
  }
  FP_(dbl)(&rr, &rr);
  FP_(sqr)(&HH, &H);
  FP_(dbl)(&I, &HH); FP_(dbl)(&I, &I);
  FP_(mul)(&J, &H, &I);
  FP_(mul)(&V, &p->x, &I);
  FP_(sqr)(&X3, &rr); FP_(sub)(&X3, &X3, &J); FP_(dbl)(&t, &V); FP_(sub)(&X3, &X3, &t);
  FP_(sub)(&t, &V, &X3); FP_(mul)(&Y3, &rr, &t);
  FP_(mul)(&t, &p->y, &J); FP_(dbl)(&t, &t); FP_(sub)(&Y3, &Y3, &t);
  FP_(add)(&Z3, &p->z, &H); FP_(sqr)(&Z3, &Z3); FP_(sub)(&Z3, &Z3, &Z1Z1); FP_(sub)(&Z3, &Z3, &HH);
  r->x = X3; r->y = Y3; r->z = Z3;
}

static void C_(jac_add)(C_(jac)* r, const C_(jac)* p, const C_(jac)* q) {
  if (C_(jac_is_inf)(p)) { *r = *q; return; }
  if (C_(jac_is_inf)(q)) { *r = *p; return; }
  FP Z1Z1, Z2Z2, U1, U2, S1, S2, H, I, J, rr, V, t, X3, Y3, Z3;
  FP_(sqr)(&Z1Z1, &p->z); FP_(sqr)(&Z2Z2, &q->z);
  FP_(mul)(&U1, &p->x, &Z2Z2); FP_(mul)(&U2, &q->x, &Z1Z1);
  FP_(mul)(&S1, &p->y, &q->z); FP_(mul)(&S1, &S1, &Z2Z2);
  FP_(mul)(&S2, &q->y, &p->z); FP_(mul)(&S2, &S2, &Z1Z1);
  FP_(sub)(&H, &U2, &U1); FP_(sub)(&rr, &S2, &S1);
  if (FP_(is_zero)(&H)) {
    if (FP_(is_zero)(&rr)) { C_(jac_dbl)(r, p); return; }
    C_(jac_set_inf)(r); return;
  }
  FP_(dbl)(&rr, &rr);
  FP_(dbl)(&I, &H); FP_(sqr)(&I, &I);
  FP_(mul)(&J, &H, &I);
  FP_(mul)(&V, &U1, &I);
  FP_(sqr)(&X3, &rr); FP_(sub)(&X3, &X3, &J); FP_(dbl)(&t, &V); FP_(sub)(&X3, &X3, &t);
  FP_(sub)(&t, &V, &X3); FP_(mul)(&Y3, &rr, &t);
  FP_(mul)(&t, &S1, &J); FP_(dbl)(&t, &t); FP_(sub)(&Y3, &Y3, &t);
  FP_(add)(&Z3, &p->z, &q->z); FP_(sqr)(&Z3, &Z3); FP_(sub)(&Z3, &Z3, &Z1Z1); FP_(sub)(&Z3, &Z3, &Z2Z2);
  FP_(mul)(&Z3, &Z3, &H);
  r->x = X3; r->y = Y3; r->z = Z3;
}

static void C_(jac_to_aff)(C_(aff)* r, const C_(jac)* p) {
  if (C_(jac_is_inf)(p)) { memset(r, 0, sizeof(*r)); r->inf = 1; return; }
  FP zi, zi2, zi3;
  FP_(inv)(&zi, &p->z); FP_(sqr)(&zi2, &zi); FP_(mul)(&zi3, &zi2, &zi);
  FP_(mul)(&r->x, &p->x, &zi2); FP_(mul)(&r->y, &p->y, &zi3); r->inf = 0;
}

static inline void C_(aff_neg)(C_(aff)* r, const C_(aff)* a) { *r = *a; if (!a->inf) FP_(neg)(&r->y, &a->y); }

static int C_(aff_on_curve)(const C_(aff)* a) {
  if (a->inf) return 1;
  FP l, rr, b; uint64_t raw[sizeof(FP) / 8];
  memset(raw, 0, sizeof(raw)); raw[0] = B_SMALL; FP_(to_mont)(&b, raw);
  FP_(sqr)(&l, &a->y);
  FP_(sqr)(&rr, &a->x); FP_(mul)(&rr, &rr, &a->x); FP_(add)(&rr, &rr, &b);
  return FP_(eq)(&l, &rr);
}

static void C_(generator)(C_(aff)* g) {
  FP_(to_mont)(&g->x, G1X); FP_(to_mont)(&g->y, G1Y); g->inf = 0;
}

/* ------------------------------------------------------------------ encodings */
static int C_(g1_decode)(C_(aff)* r, const uint8_t* b) {
  memset(r, 0, sizeof(*r));
#if IS_BLS
  uint8_t f = b[0] & 0xE0;
  if (f & 0x80) return KZGO_ERR_ENCODING;
  if (f & 0x40) {
    if (b[0] & 0x3F) return KZGO_ERR_ENCODING;
    for (int i = 1; i < 2 * FPB; ++i) if (b[i]) return KZGO_ERR_ENCODING;
    r->inf = 1; return 0;
  }
  if (f & 0x20) return KZGO_ERR_ENCODING;
#else
  int allz = 1;
  for (int i = 0; i < 2 * FPB; ++i) if (b[i]) { allz = 0; break; }
  if (allz) { r->inf = 1; return 0; }
#endif
  if (FP_(from_be)(&r->x, b, FPB)) return KZGO_ERR_ENCODING;
  if (FP_(from_be)(&r->y, b + FPB, FPB)) return KZGO_ERR_ENCODING;
  if (!C_(aff_on_curve)(r)) return KZGO_ERR_NOT_ON_CURVE;
  return 0;
}
static void C_(g1_encode)(uint8_t* b, const C_(aff)* a) {
  memset(b, 0, 2 * FPB);
  if (a->inf) {
#if IS_BLS
    b[0] = 0x40;
#endif
    return;
  }
  FP_(to_be)(b, &a->x, FPB); FP_(to_be)(b + FPB, &a->y, FPB);
}

static int C_(g2_on_curve)(const C_(aff2)* a) {
  if (a->inf) return 1;
  T_(fp2) l, rr, b2;
  FP_(to_mont)(&b2.c0, B2_0); FP_(to_mont)(&b2.c1, B2_1);
  T_(fp2_mul)(&l, &a->y, &a->y);
  T_(fp2_mul)(&rr, &a->x, &a->x); T_(fp2_mul)(&rr, &rr, &a->x); T_(fp2_add)(&rr, &rr, &b2);
  return T_(fp2_eq)(&l, &rr);
}
static int C_(g2_decode)(C_(aff2)* r, const uint8_t* b) {
  memset(r, 0, sizeof(*r));
#if IS_BLS
  if (b[0] & 0x80) return KZGO_ERR_ENCODING;
  if (b[0] & 0x40) { r->inf = 1; return 0; }
#else
  int allz = 1;
  for (int i = 0; i < 4 * FPB; ++i) if (b[i]) { allz = 0; break; }
  if (allz) { r->inf = 1; return 0; }
#endif
  if (FP_(from_be)(&r->x.c1, b, FPB) || FP_(from_be)(&r->x.c0, b + FPB, FPB) ||
      FP_(from_be)(&r->y.c1, b + 2 * FPB, FPB) || FP_(from_be)(&r->y.c0, b + 3 * FPB, FPB))
    return KZGO_ERR_ENCODING;
  if (!C_(g2_on_curve)(r)) return KZGO_ERR_NOT_ON_CURVE;
  return 0;
}
static void C_(g2_encode)(uint8_t* b, const C_(aff2)* a) {
  memset(b, 0, 4 * FPB);
  if (a->inf) {
#if IS_BLS
    b[0] = 0x40;
#endif
    return;
  }
  FP_(to_be)(b, &a->x.c1, FPB); FP_(to_be)(b + FPB, &a->x.c0, FPB);
  FP_(to_be)(b + 2 * FPB, &a->y.c1, FPB); FP_(to_be)(b + 3 * FPB, &a->y.c0, FPB);
}

/* scalar: 32 bytes BE, canonical (< r) -> raw 4x64 */
static int C_(fr_decode_raw)(uint64_t* raw, const uint8_t* b) {
  FR_(raw_from_be)(raw, b, 32);
  return FR_(geq_mod)(raw) ? KZGO_ERR_SCALAR : 0;
}

/* ------------------------------------------------------------------ compressed G1 */
/* BLS12-381: 48 B ZCash flags (0x80 compressed, 0x40 infinity, 0x20 larger y);
 * BN254: 32 B gnark-crypto (top bits 0b10 smaller y, 0b11 larger y, 0b01 infinity). */
static int C_(y_is_larger)(const FP* y) {  /* raw y > (p-1)/2 <=> 2y > p - 1 <=> 2y >= p */
  uint64_t raw[sizeof(FP) / 8]; FP_(from_mont)(raw, y);
  uint64_t dbl[sizeof(FP) / 8 + 1]; uint64_t c = 0;
  for (size_t i = 0; i < sizeof(FP) / 8; ++i) { dbl[i] = (raw[i] << 1) | c; c = raw[i] >> 63; }
  if (c) return 1;
  for (int i = (int)(sizeof(FP) / 8) - 1; i >= 0; --i) {
    if (dbl[i] != PRAW[i]) return dbl[i] > PRAW[i];
  }
  return 1;  /* 2y == p impossible (p odd) */
}
static int C_(g1_decode_compressed)(C_(aff)* r, const uint8_t* b) {
  memset(r, 0, sizeof(*r));
  uint8_t xb[FPB]; memcpy(xb, b, FPB);
  int larger;
  int rest = 0;
  for (int i = 1; i < FPB; ++i) rest |= b[i];
#if IS_BLS
  if (!(b[0] & 0x80)) return KZGO_ERR_ENCODING;
  if (b[0] & 0x40) { if (b[0] != 0xC0 || rest) return KZGO_ERR_ENCODING; r->inf = 1; return 0; }
  larger = (b[0] & 0x20) != 0;
  xb[0] &= 0x1F;
#else
  uint8_t m = b[0] & 0xC0;
  if (m == 0x40) { if (b[0] != 0x40 || rest) return KZGO_ERR_ENCODING; r->inf = 1; return 0; }
  if (m == 0x00) return KZGO_ERR_ENCODING;
  larger = m == 0xC0;
  xb[0] &= 0x3F;
#endif
  if (FP_(from_be)(&r->x, xb, FPB)) return KZGO_ERR_ENCODING;
  FP rhs, bb, y, y2; uint64_t raw[sizeof(FP) / 8];
  memset(raw, 0, sizeof(raw)); raw[0] = B_SMALL; FP_(to_mont)(&bb, raw);
  FP_(sqr)(&rhs, &r->x); FP_(mul)(&rhs, &rhs, &r->x); FP_(add)(&rhs, &rhs, &bb);
  uint64_t e[sizeof(FP) / 8]; uint64_t c = 1;  /* e = (p + 1) / 4 */
  for (size_t i = 0; i < sizeof(FP) / 8; ++i) { uint64_t t = PRAW[i] + c; c = t < c; e[i] = t; }
  for (size_t i = 0; i < sizeof(FP) / 8; ++i) e[i] = (e[i] >> 2) | (i + 1 < sizeof(FP) / 8 ? e[i + 1] << 62 : 0);
  FP_(pow)(&y, &rhs, e, (int)(sizeof(FP) * 8));
  FP_(sqr)(&y2, &y);
  if (!FP_(eq)(&y2, &rhs)) return KZGO_ERR_NOT_ON_CURVE;
  if (FP_(is_zero)(&y) && larger) return KZGO_ERR_ENCODING;
  if (C_(y_is_larger)(&y) != larger) FP_(neg)(&y, &y);
  r->y = y;
  return 0;
}
static void C_(g1_encode_compressed)(uint8_t* b, const C_(aff)* a) {
  memset(b, 0, FPB);
#if IS_BLS
  if (a->inf) { b[0] = 0xC0; return; }
  FP_(to_be)(b, &a->x, FPB);
  b[0] |= 0x80 | (C_(y_is_larger)(&a->y) ? 0x20 : 0);
#else
  if (a->inf) { b[0] = 0x40; return; }
  FP_(to_be)(b, &a->x, FPB);
  b[0] |= C_(y_is_larger)(&a->y) ? 0xC0 : 0x80;
#endif
}

/* ------------------------------------------------------------------ scalar mul */
static inline int C_(bit)(const uint64_t* k, int i) { return (int)((k[i >> 6] >> (i & 63)) & 1); }

static void C_(mul_raw)(C_(jac)* r, const C_(aff)* p, const uint64_t* k) {
  C_(jac) acc; C_(jac_set_inf)(&acc);
  for (int i = 255; i >= 0; --i) {
    C_(jac_dbl)(&acc, &acc);
    if (C_(bit)(k, i)) C_(jac_add_aff)(&acc, &acc, p);
  }
  *r = acc;
}

/* subgroup membership by definition: [r]P == O */
static int C_(in_subgroup)(const C_(aff)* p) {
  if (p->inf) return 1;
  C_(jac) q; C_(mul_raw)(&q, p, RRAW);
  return C_(jac_is_inf)(&q);
}

/* ------------------------------------------------------------------ Pippenger */
static inline unsigned C_(window)(const uint64_t* k, int start, int c) {
  unsigned v = 0;
  for (int b = 0; b < c; ++b) {
    int i = start + b;
    if (i < 256 && C_(bit)(k, i)) v |= 1u << b;
  }
  return v;
}

static void C_(msm_chunk)(C_(jac)* out, const C_(aff)* pts, const uint64_t* sc, size_t n) {
  C_(jac_set_inf)(out);
  if (n == 0) return;
  int lg = 0; while (((size_t)1 << (lg + 1)) <= n) ++lg;
  int c = lg - 2; if (c < 2) c = 2; if (c > 16) c = 16;
  int nw = (256 + c - 1) / c;
  size_t nb = ((size_t)1 << c) - 1;
  C_(jac)* buckets = (C_(jac)*)malloc(nb * sizeof(C_(jac)));
  C_(jac) total; C_(jac_set_inf)(&total);
  for (int w = nw - 1; w >= 0; --w) {
    for (int d = 0; d < c; ++d) C_(jac_dbl)(&total, &total);
    for (size_t b = 0; b < nb; ++b) C_(jac_set_inf)(&buckets[b]);
    for (size_t i = 0; i < n; ++i) {
      unsigned d = C_(window)(sc + 4 * i, w * c, c);
      if (d && !pts[i].inf) C_(jac_add_aff)(&buckets[d - 1], &buckets[d - 1], &pts[i]);
    }
    C_(jac) run, sum; C_(jac_set_inf)(&run); C_(jac_set_inf)(&sum);
    for (size_t b = nb; b-- > 0;) {
      C_(jac_add)(&run, &run, &buckets[b]);
      C_(jac_add)(&sum, &sum, &run);
    }
    C_(jac_add)(&total, &total, &sum);
  }
  free(buckets);
  *out = total;
}

static void C_(msm)(C_(jac)* out, const C_(aff)* pts, const uint64_t* sc, size_t n) {
  int nt = kzgo_threads();
  if ((size_t)nt > n / 64 + 1) nt = (int)(n / 64 + 1);
  C_(jac)* part = (C_(jac)*)malloc((size_t)nt * sizeof(C_(jac)));
  #pragma omp parallel for num_threads(nt) schedule(static)
  for (int t = 0; t < nt; ++t) {
    size_t lo = n * (size_t)t / nt, hi = n * (size_t)(t + 1) / nt;
    C_(msm_chunk)(&part[t], pts + lo, sc + 4 * lo, hi - lo);
  }
  C_(jac) acc; C_(jac_set_inf)(&acc);
  for (int t = 0; t < nt; ++t) C_(jac_add)(&acc, &acc, &part[t]);
  free(part);
  *out = acc;
}

/* ------------------------------------------------------------------ pairing */
/* Sparse line for T (affine twist) with slope lam, evaluated at P (affine, Fp), written as
 * a full Fp12 (then multiplied with the schoolbook Fp12 product).
 *  M-type (times w^3): (yT - lam xT) + (lam xP) w^2 - yP w^3
 *  D-type:             -yP + (lam xP) w + (yT - lam xT) w^3                              */
static void C_(line)(T_(fp12)* l, const C_(aff2)* T, const T_(fp2)* lam, const C_(aff)* P) {
  memset(l, 0, sizeof(*l));
  T_(fp2) a, b, c;
  T_(fp2_mul)(&a, lam, &T->x); T_(fp2_sub)(&a, &T->y, &a);   /* yT - lam xT */
  T_(fp2_mul_fp)(&b, lam, &P->x);                            /* lam xP */
  T_(fp2_zero)(&c); FP_(neg)(&c.c0, &P->y);                  /* -yP */
#if IS_BLS
  l->c0.c0 = a; l->c0.c1 = b; l->c1.c1 = c;
#else
  l->c0.c0 = c; l->c1.c0 = b; l->c1.c1 = a;
#endif
}
static void C_(vertical)(T_(fp12)* l, const C_(aff2)* T, const C_(aff)* P) {
  memset(l, 0, sizeof(*l));
  T_(fp2) xp, nx; T_(fp2_zero)(&xp); xp.c0 = P->x; T_(fp2_neg)(&nx, &T->x);
#if IS_BLS
  l->c0.c0 = nx; l->c0.c1 = xp;   /* (xP - xT w^-2) w^2 */
#else
  l->c0.c0 = xp; l->c0.c1 = nx;   /*  xP - xT w^2       */
#endif
}
/* f *= line(T, Q)(P); T += Q  (Q == T means doubling) */
static void C_(step)(T_(fp12)* f, C_(aff2)* T, const C_(aff2)* Q, const C_(aff)* P) {
  if (T->inf) { *T = *Q; return; }
  if (Q->inf) return;
  T_(fp2) lam, t, u;
  if (T_(fp2_eq)(&T->x, &Q->x)) {
    T_(fp2_add)(&t, &T->y, &Q->y);
    if (T_(fp2_is_zero)(&t)) {
      T_(fp12) l; C_(vertical)(&l, T, P); T_(fp12_mul)(f, f, &l);
      memset(T, 0, sizeof(*T)); T->inf = 1; return;
    }
    T_(fp2_mul)(&t, &T->x, &T->x); T_(fp2_add)(&u, &t, &t); T_(fp2_add)(&t, &u, &t); /* 3x^2 */
    T_(fp2_add)(&u, &T->y, &T->y); T_(fp2_inv)(&u, &u); T_(fp2_mul)(&lam, &t, &u);
  } else {
    T_(fp2_sub)(&t, &Q->y, &T->y); T_(fp2_sub)(&u, &Q->x, &T->x);
    T_(fp2_inv)(&u, &u); T_(fp2_mul)(&lam, &t, &u);
  }
  T_(fp12) l; C_(line)(&l, T, &lam, P); T_(fp12_mul)(f, f, &l);
  T_(fp2) x3, y3;
  T_(fp2_mul)(&x3, &lam, &lam); T_(fp2_sub)(&x3, &x3, &T->x); T_(fp2_sub)(&x3, &x3, &Q->x);
  T_(fp2_sub)(&t, &T->x, &x3); T_(fp2_mul)(&y3, &lam, &t); T_(fp2_sub)(&y3, &y3, &T->y);
  T->x = x3; T->y = y3;
}

static void C_(frob_twist)(C_(aff2)* r, const C_(aff2)* q) {
  T_(fp2) gx, gy, xc, yc;
  FP_(to_mont)(&gx.c0, FROB_GX0); FP_(to_mont)(&gx.c1, FROB_GX1);
  FP_(to_mont)(&gy.c0, FROB_GY0); FP_(to_mont)(&gy.c1, FROB_GY1);
  T_(fp2_conj)(&xc, &q->x); T_(fp2_conj)(&yc, &q->y);
  T_(fp2_mul)(&r->x, &xc, &gx); T_(fp2_mul)(&r->y, &yc, &gy); r->inf = q->inf;
}

static void C_(miller)(T_(fp12)* f, const C_(aff)* P, const C_(aff2)* Q) {
  T_(fp12_one)(f);
  if (P->inf || Q->inf) return;
  C_(aff2) T = *Q;
  for (int i = LOOP_BITS - 2; i >= 0; --i) {
    T_(fp12_mul)(f, f, f);
    C_(aff2) Tc = T;
    C_(step)(f, &T, &Tc, P);
    if ((LOOP_WORDS[i / 64] >> (i % 64)) & 1) C_(step)(f, &T, Q, P);
  }
#if IS_BLS
  T_(fp12_conj)(f, f);
#else
  C_(aff2) Q1, Q2;
  C_(frob_twist)(&Q1, Q);
  C_(frob_twist)(&Q2, &Q1);
  T_(fp2_neg)(&Q2.y, &Q2.y);
  C_(step)(f, &T, &Q1, P);
  C_(step)(f, &T, &Q2, P);
#endif
}

static void C_(final_exp)(T_(fp12)* r, const T_(fp12)* f) {
  T_(fp12_pow)(r, f, FEXP, FEXP_BITS);
}

static void C_(fp12_encode)(uint8_t* out, const T_(fp12)* f) {
  const FP* c[12] = {&f->c0.c0.c0, &f->c0.c0.c1, &f->c0.c1.c0, &f->c0.c1.c1, &f->c0.c2.c0, &f->c0.c2.c1,
                     &f->c1.c0.c0, &f->c1.c0.c1, &f->c1.c1.c0, &f->c1.c1.c1, &f->c1.c2.c0, &f->c1.c2.c1};
  for (int i = 0; i < 12; ++i) FP_(to_be)(out + i * FPB, c[i], FPB);
}

/* ------------------------------------------------------------------ batch verify */
/* pairing check e(A, [tau]_2) * e(-B, [1]_2) == 1 for given affine A, B */
static void C_(pairing_check)(const C_(aff)* A, const C_(aff)* B, const C_(aff2)* g2, const C_(aff2)* tg2, int* ok) {
  C_(aff) nB;
  C_(aff_neg)(&nB, B);
  T_(fp12) f1, f2, f;
  C_(miller)(&f1, A, tg2);
  C_(miller)(&f2, &nB, g2);
  T_(fp12_mul)(&f, &f1, &f2);
  C_(final_exp)(&f, &f);
  *ok = T_(fp12_is_one)(&f);
}

/* offset = global index of tuple 0 (shards); do_pairing = 0 only computes A, B */
/* seed != NULL: r_i = randomizer(seed, offset + i) (127-bit); pow_r != NULL (32 B big-endian r < r):
 * r_i = r^(offset + i) (Fiat-Shamir / powers mode). */
static int C_(batch_verify)(const uint8_t* cm, const uint8_t* zs, const uint8_t* ys, const uint8_t* pf,
                            size_t n, const uint8_t* g2b, const uint8_t* tg2b, const uint8_t* seed,
                            int* ok, uint8_t* a_out, uint8_t* b_out, uint64_t offset, int do_pairing,
                            const uint8_t* pow_r, const uint8_t* g1b) {
  C_(aff2) g2, tg2;
  C_(aff) g1;
  int e;
  if ((e = C_(g2_decode)(&g2, g2b))) return e;
  if ((e = C_(g2_decode)(&tg2, tg2b))) return e;
  if (g1b) {  /* the SRS's [1]_1 (SURVEY.md 8b srs = {G1, [1]_2, [tau]_2}); NULL = the standard generator */
    if ((e = C_(g1_decode)(&g1, g1b))) return e;
  } else {
    C_(generator)(&g1);
  }
  if (n == 0) {
    *ok = 1;
    C_(aff) inf; memset(&inf, 0, sizeof(inf)); inf.inf = 1;
    if (a_out) C_(g1_encode)(a_out, &inf);
    if (b_out) C_(g1_encode)(b_out, &inf);
    return 0;
  }
  C_(aff)* pts = (C_(aff)*)malloc((2 * n + 1) * sizeof(C_(aff)));   /* [C..., pi..., G] */
  uint64_t* sc = (uint64_t*)malloc((2 * n + 1) * 4 * sizeof(uint64_t)); /* [r..., s..., -t] */
  int err = 0;
  FR tsum; FR_(zero)(&tsum);
  FR rbase;  /* powers mode: r in Montgomery form */
  if (pow_r) {
    uint64_t raw[4];
    if ((e = C_(fr_decode_raw)(raw, pow_r))) { free(pts); free(sc); return e; }
    FR_(to_mont)(&rbase, raw);
  }
  #pragma omp parallel num_threads(kzgo_threads())
  {
    FR tloc; FR_(zero)(&tloc);
    const size_t nt = (size_t)omp_get_num_threads(), tid = (size_t)omp_get_thread_num();
    const size_t lo = n * tid / nt, hi = n * (tid + 1) / nt;
    FR rcur;  /* powers mode: r^(offset + i), stepped by r */
    if (pow_r) {
      uint64_t ex[1] = {offset + (uint64_t)lo};
      FR_(pow)(&rcur, &rbase, ex, 64);
    }
    for (size_t i = lo; i < hi; ++i) {
      int le = C_(g1_decode)(&pts[i], cm + i * 2 * FPB);
      if (!le) le = C_(g1_decode)(&pts[n + i], pf + i * 2 * FPB);
      uint64_t z[4], y[4], ri[4];
      if (!le) le = C_(fr_decode_raw)(z, zs + 32 * i);
      if (!le) le = C_(fr_decode_raw)(y, ys + 32 * i);
      if (le) {
        #pragma omp critical
        { if (!err) err = le; }
        continue;
      }
      FR rm, zm, ym, s;
      if (pow_r) {
        rm = rcur;
        FR_(mul)(&rcur, &rcur, &rbase);
        FR_(from_mont)(ri, &rm);
      } else {
        kzgo_randomizer(seed, offset + (uint64_t)i, ri);
        FR_(to_mont)(&rm, ri);
      }
      memcpy(sc + 4 * i, ri, 32);
      FR_(to_mont)(&zm, z); FR_(to_mont)(&ym, y);
      FR_(mul)(&s, &rm, &zm); FR_(from_mont)(sc + 4 * (n + i), &s);
      FR_(mul)(&s, &rm, &ym); FR_(add)(&tloc, &tloc, &s);
    }
    #pragma omp critical
    FR_(add)(&tsum, &tsum, &tloc);
  }
  if (err) { free(pts); free(sc); return err; }
  pts[2 * n] = g1;
  FR nt; FR_(neg)(&nt, &tsum); FR_(from_mont)(sc + 4 * (2 * n), &nt);
  /* A = sum r_i pi_i ; B = sum r_i C_i + s_i pi_i - t G */
  uint64_t* sa = (uint64_t*)malloc(n * 4 * sizeof(uint64_t));
  memcpy(sa, sc, n * 32);
  C_(jac) Aj, Bj;
  C_(msm)(&Aj, pts + n, sa, n);
  C_(msm)(&Bj, pts, sc, 2 * n + 1);
  free(sa); free(pts); free(sc);
  C_(aff) A, B, nB;
  C_(jac_to_aff)(&A, &Aj); C_(jac_to_aff)(&B, &Bj);
  if (a_out) C_(g1_encode)(a_out, &A);
  if (b_out) C_(g1_encode)(b_out, &B);
  (void)nB;
  *ok = -1;
  if (do_pairing) C_(pairing_check)(&A, &B, &g2, &tg2, ok);
  return 0;
}

static int C_(pairing_check_api)(const uint8_t* a, const uint8_t* b, const uint8_t* g2b, const uint8_t* tg2b, int* ok) {
  C_(aff) A, B; C_(aff2) g2, tg2; int e;
  if ((e = C_(g1_decode)(&A, a)) || (e = C_(g1_decode)(&B, b))) return e;
  if ((e = C_(g2_decode)(&g2, g2b)) || (e = C_(g2_decode)(&tg2, tg2b))) return e;
  C_(pairing_check)(&A, &B, &g2, &tg2, ok);
  return 0;
}
