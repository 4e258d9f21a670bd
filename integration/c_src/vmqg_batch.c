/*
 * vmqg_batch.c — see vmqg_batch.h.  Plain C99, no OTP, no HIP: only the
 * libvmqgpu C ABI.
 */
#define _POSIX_C_SOURCE 200809L   /* clock_gettime under -std=c99 */
#include "vmqg_batch.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static uint64_t mono_ns(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

/* ------------------------------------------------------------ interner */
/* Open addressing over (hash, id + 1); an erased slot holds ERASED and
 * probes continue past it.  Keys live back to back in `bytes` (offs / lens
 * per id); a removed key's bytes are garbage until the buffer is packed.
 * Ids removed and then released are reused, lowest-released first out. */
#define ERASED 0xFFFFFFFFu
struct vmqgb_interner {
  uint8_t* bytes;       /* every key, back to back */
  size_t nbytes, bcap, garbage;
  uint64_t* offs;       /* id -> start in bytes */
  uint32_t* lens;       /* id -> length; ERASED: not a live key */
  uint32_t n, ocap;     /* ids handed out: [0, n) */
  uint32_t live, erased;
  uint32_t* slots;      /* open addressing: id + 1, 0 = empty, ERASED = erased */
  uint64_t* hashes;     /* per slot */
  uint32_t mask;
  uint32_t* free_ids;   /* released ids */
  uint32_t nfree, fcap;
};

static uint64_t hash_bytes(const void* p, size_t len) {   /* FNV-1a, then a 64-bit finaliser */
  const uint8_t* b = (const uint8_t*)p;
  uint64_t h = 0xcbf29ce484222325ull;
  for (size_t i = 0; i < len; i++) { h ^= b[i]; h *= 0x100000001b3ull; }
  h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33;
  return h;
}

vmqgb_interner* vmqgb_interner_new(void) {
  vmqgb_interner* t = (vmqgb_interner*)calloc(1, sizeof(*t));
  if (!t) return NULL;
  t->mask = 1023;
  t->slots = (uint32_t*)calloc(1024, sizeof(uint32_t));
  t->hashes = (uint64_t*)calloc(1024, sizeof(uint64_t));
  t->ocap = 1024;
  t->offs = (uint64_t*)calloc(t->ocap, sizeof(uint64_t));
  t->lens = (uint32_t*)calloc(t->ocap, sizeof(uint32_t));
  if (!t->slots || !t->hashes || !t->offs || !t->lens) { vmqgb_interner_free(t); return NULL; }
  return t;
}

void vmqgb_interner_free(vmqgb_interner* t) {
  if (!t) return;
  free(t->bytes); free(t->offs); free(t->lens); free(t->slots); free(t->hashes); free(t->free_ids); free(t);
}

static int eq_at(const vmqgb_interner* t, uint32_t id, const void* bytes, size_t len) {
  return t->lens[id] == len && memcmp(t->bytes + t->offs[id], bytes, len) == 0;
}

static void rehash(vmqgb_interner* t, uint32_t ncap) {
  uint32_t* s = (uint32_t*)calloc(ncap, sizeof(uint32_t));
  uint64_t* h = (uint64_t*)calloc(ncap, sizeof(uint64_t));
  if (!s || !h) { free(s); free(h); return; }   /* keeps the old table: still correct, only fuller */
  for (uint32_t i = 0; i <= t->mask; i++) {
    if (!t->slots[i] || t->slots[i] == ERASED) continue;
    uint32_t j = (uint32_t)t->hashes[i] & (ncap - 1);
    while (s[j]) j = (j + 1) & (ncap - 1);
    s[j] = t->slots[i];
    h[j] = t->hashes[i];
  }
  free(t->slots); free(t->hashes);
  t->slots = s; t->hashes = h; t->mask = ncap - 1;
  t->erased = 0;
}

/* the live keys packed to the front of a fresh buffer (removed keys' bytes dropped) */
static void pack(vmqgb_interner* t) {
  uint8_t* nb = (uint8_t*)malloc(t->nbytes - t->garbage + 1);
  if (!nb) return;
  size_t o = 0;
  for (uint32_t id = 0; id < t->n; id++) {
    if (t->lens[id] == ERASED) continue;
    memcpy(nb + o, t->bytes + t->offs[id], t->lens[id]);
    t->offs[id] = o;
    o += t->lens[id];
  }
  free(t->bytes);
  t->bytes = nb;
  t->bcap = t->nbytes - t->garbage + 1;
  t->nbytes = o;
  t->garbage = 0;
}

int vmqgb_lookup(const vmqgb_interner* t, const void* bytes, size_t len, uint32_t* id) {
  const uint64_t hv = hash_bytes(bytes, len);
  for (uint32_t j = (uint32_t)hv & t->mask;; j = (j + 1) & t->mask) {
    const uint32_t v = t->slots[j];
    if (!v) return -1;
    if (v != ERASED && t->hashes[j] == hv && eq_at(t, v - 1, bytes, len)) { if (id) *id = v - 1; return 0; }
  }
}

uint32_t vmqgb_intern(vmqgb_interner* t, const void* bytes, size_t len) { return vmqgb_intern_ex(t, bytes, len, NULL); }

uint32_t vmqgb_intern_ex(vmqgb_interner* t, const void* bytes, size_t len, int* created) {
  const uint64_t hv = hash_bytes(bytes, len);
  uint32_t j = (uint32_t)hv & t->mask;
  if (created) *created = 0;
  for (;; j = (j + 1) & t->mask) {
    const uint32_t v = t->slots[j];
    if (!v) break;
    if (v != ERASED && t->hashes[j] == hv && eq_at(t, v - 1, bytes, len)) return v - 1;
  }
  if (created) *created = 1;
  if (len >= ERASED) return VMQG_NONE;
  if (t->nbytes + len > t->bcap) {
    size_t c = t->bcap ? t->bcap * 2 : 4096;
    while (c < t->nbytes + len) c *= 2;
    uint8_t* nb = (uint8_t*)realloc(t->bytes, c);
    if (!nb) return VMQG_NONE;
    t->bytes = nb; t->bcap = c;
  }
  uint32_t id;
  if (t->nfree) {
    id = t->free_ids[--t->nfree];
  } else {
    if (t->n + 1 >= t->ocap) {
      uint64_t* no = (uint64_t*)realloc(t->offs, (size_t)t->ocap * 2 * sizeof(uint64_t));
      if (!no) return VMQG_NONE;
      t->offs = no;
      uint32_t* nl = (uint32_t*)realloc(t->lens, (size_t)t->ocap * 2 * sizeof(uint32_t));
      if (!nl) return VMQG_NONE;
      t->lens = nl;
      t->ocap *= 2;
    }
    id = t->n++;
  }
  if (len) memcpy(t->bytes + t->nbytes, bytes, len);
  t->offs[id] = t->nbytes;
  t->lens[id] = (uint32_t)len;
  t->nbytes += len;
  t->slots[j] = id + 1;
  t->hashes[j] = hv;
  t->live++;
  if ((uint64_t)(t->live + t->erased) * 2 > t->mask + 1) rehash(t, (uint64_t)t->live * 4 > t->mask + 1 ? (t->mask + 1) * 2 : t->mask + 1);
  return id;
}

int vmqgb_interner_remove(vmqgb_interner* t, uint32_t id) {
  if (id >= t->n || t->lens[id] == ERASED) return -1;
  const uint64_t hv = hash_bytes(t->bytes + t->offs[id], t->lens[id]);
  for (uint32_t j = (uint32_t)hv & t->mask;; j = (j + 1) & t->mask) {
    const uint32_t v = t->slots[j];
    if (!v) return -1;
    if (v == id + 1) { t->slots[j] = ERASED; break; }
  }
  t->garbage += t->lens[id];
  t->lens[id] = ERASED;
  t->live--;
  t->erased++;
  if (t->garbage > 4096 && t->garbage * 2 > t->nbytes) pack(t);
  return 0;
}

int vmqgb_interner_release(vmqgb_interner* t, uint32_t id) {
  if (id >= t->n || t->lens[id] != ERASED) return -1;
  if (t->nfree == t->fcap) {
    const uint32_t c = t->fcap ? t->fcap * 2 : 1024;
    uint32_t* nf = (uint32_t*)realloc(t->free_ids, (size_t)c * sizeof(uint32_t));
    if (!nf) return -1;   /* the id stays unused: only memory */
    t->free_ids = nf;
    t->fcap = c;
  }
  t->free_ids[t->nfree++] = id;
  return 0;
}

const uint8_t* vmqgb_bytes(const vmqgb_interner* t, uint32_t id, size_t* len) {
  if (id >= t->n || t->lens[id] == ERASED) return NULL;
  if (len) *len = t->lens[id];
  return t->bytes + t->offs[id];
}

uint32_t vmqgb_count(const vmqgb_interner* t) { return t->n; }
uint32_t vmqgb_live(const vmqgb_interner* t) { return t->live; }

/* -------------------------------------------------------------- batches */
static int grow(void** p, size_t* cap, size_t need, size_t esz) {
  if (need <= *cap) return 0;
  size_t c = *cap ? *cap : 64;
  while (c < need) c *= 2;
  void* np = realloc(*p, c * esz);
  if (!np) return VMQG_E_NOMEM;
  *p = np;
  *cap = c;
  return 0;
}

int vmqgb_batch_init(vmqgb_batch* b, size_t cap_hint) {
  memset(b, 0, sizeof(*b));
  if (cap_hint < 64) cap_hint = 64;
  if (grow((void**)&b->pubs, &b->cap, cap_hint, sizeof(vmqg_pub))) return VMQG_E_NOMEM;
  if (grow((void**)&b->words, &b->wcap, cap_hint * 4, sizeof(uint32_t))) return VMQG_E_NOMEM;
  return 0;
}

void vmqgb_batch_reset(vmqgb_batch* b) {
  b->n = b->nwords = b->out_n = b->rng_n = 0;
  b->n_unk = b->raw_n = 0;
  b->dict_gen = 0;
}

void vmqgb_batch_free(vmqgb_batch* b) {
  free(b->pubs); free(b->words); free(b->offs_buf); free(b->out); free(b->rng_buf);
  free(b->unk); free(b->raw);
  memset(b, 0, sizeof(*b));
}

/* remembers publish i's raw topic when it holds a word the dictionary did not know */
static int note_unknown(vmqgb_batch* b, size_t i, const uint8_t* topic, size_t len) {
  if (grow((void**)&b->unk, &b->unk_cap, 3 * (b->n_unk + 1), sizeof(uint32_t))) return VMQG_E_NOMEM;
  if (grow((void**)&b->raw, &b->raw_cap, b->raw_n + len, 1)) return VMQG_E_NOMEM;
  memcpy(b->raw + b->raw_n, topic, len);
  b->unk[3 * b->n_unk] = (uint32_t)i;
  b->unk[3 * b->n_unk + 1] = (uint32_t)b->raw_n;
  b->unk[3 * b->n_unk + 2] = (uint32_t)len;
  b->n_unk++;
  b->raw_n += len;
  return 0;
}

long vmqgb_batch_add(vmqgb_batch* b, vmqg_ctx* ctx, uint32_t mountpoint, const uint8_t* topic, size_t len) {
  if (grow((void**)&b->pubs, &b->cap, b->n + 1, sizeof(vmqg_pub))) return VMQG_E_NOMEM;
  if (b->n == 0) b->dict_gen = vmqg_dict_generation(ctx);
  /* a topic of len bytes has at most len + 1 words */
  size_t room = b->wcap - b->nwords;
  if (room < 16 && grow((void**)&b->words, &b->wcap, b->nwords + 16, sizeof(uint32_t))) return VMQG_E_NOMEM;
  for (;;) {
    room = b->wcap - b->nwords;
    vmqg_pub pub;
    const uint32_t cap = room > 0xFFFFFFFFu ? 0xFFFFFFFFu : (uint32_t)room;
    const int rc = vmqg_prepare_publish(ctx, mountpoint, topic, len, b->words + b->nwords, cap, &pub);
    if (rc == VMQG_E_OVERFLOW) {
      if (grow((void**)&b->words, &b->wcap, b->nwords + len + 1, sizeof(uint32_t))) return VMQG_E_NOMEM;
      continue;
    }
    if (rc) return rc;
    pub.word_off = (uint32_t)b->nwords;
    if ((pub.flags & VMQG_PUB_UNKNOWN) && note_unknown(b, b->n, topic, len)) return VMQG_E_NOMEM;
    b->nwords += pub.nwords;
    b->pubs[b->n] = pub;
    return (long)b->n++;
  }
}

int vmqgb_batch_add_many(vmqgb_batch* b, vmqg_ctx* ctx, size_t n, const uint32_t* mountpoints,
                         const uint8_t* const* topics, const size_t* lens, long* idx_out) {
  if (!n) return 0;
  if (b->n == 0) b->dict_gen = vmqg_dict_generation(ctx);
  const size_t n_unk0 = b->n_unk, raw0 = b->raw_n;   /* restored on failure: no note may name a slot past b->n */
  size_t need = 0;
  for (size_t i = 0; i < n; i++) need += lens[i] + 1;
  if (grow((void**)&b->pubs, &b->cap, b->n + n, sizeof(vmqg_pub))) return VMQG_E_NOMEM;
  if (grow((void**)&b->words, &b->wcap, b->nwords + need, sizeof(uint32_t))) return VMQG_E_NOMEM;
  int32_t stack_rc[256];
  int32_t* rcs = n <= 256 ? stack_rc : (int32_t*)malloc(n * sizeof(int32_t));
  if (!rcs) return VMQG_E_NOMEM;
  vmqg_pub* P = b->pubs + b->n;
  size_t nw = 0;
  int rc = vmqg_prepare_publishes(ctx, n, mountpoints, topics, lens, P, rcs, b->words + b->nwords, b->wcap - b->nwords, &nw);
  if (rc) { if (rcs != stack_rc) free(rcs); return rc; }
  /* compact: rejected topics take no slot in the batch */
  size_t k = b->n;
  for (size_t i = 0; i < n; i++) {
    if (rcs[i]) { idx_out[i] = rcs[i]; continue; }
    vmqg_pub pub = P[i];
    pub.word_off += (uint32_t)b->nwords;
    if ((pub.flags & VMQG_PUB_UNKNOWN) && note_unknown(b, k, topics[i], lens[i])) { rc = VMQG_E_NOMEM; break; }
    b->pubs[k] = pub;
    idx_out[i] = (long)k++;
  }
  if (rcs != stack_rc) free(rcs);
  if (rc) { b->n_unk = n_unk0; b->raw_n = raw0; return rc; }
  b->n = k;
  b->nwords += nw;
  return 0;
}

/* a word list as its unknown-word note: {u32 len, bytes} per word */
static int note_unknown_words(vmqgb_batch* b, size_t i, uint32_t cnt, const uint8_t* const* words, const size_t* lens) {
  size_t bytes = 0;
  for (uint32_t j = 0; j < cnt; j++) bytes += 4 + (lens[j] == VMQGB_NOT_BINARY ? 0 : lens[j]);
  if (bytes >= VMQGB_RAW_WORDS) return VMQG_E_NOMEM;
  if (grow((void**)&b->unk, &b->unk_cap, 3 * (b->n_unk + 1), sizeof(uint32_t))) return VMQG_E_NOMEM;
  if (grow((void**)&b->raw, &b->raw_cap, b->raw_n + bytes, 1)) return VMQG_E_NOMEM;
  uint8_t* d = b->raw + b->raw_n;
  for (uint32_t j = 0; j < cnt; j++) {
    const uint32_t l = lens[j] == VMQGB_NOT_BINARY ? 0xFFFFFFFFu : (uint32_t)lens[j];
    memcpy(d, &l, 4);
    d += 4;
    if (l != 0xFFFFFFFFu && l) { memcpy(d, words[j], l); d += l; }
  }
  b->unk[3 * b->n_unk] = (uint32_t)i;
  b->unk[3 * b->n_unk + 1] = (uint32_t)b->raw_n;
  b->unk[3 * b->n_unk + 2] = (uint32_t)bytes | VMQGB_RAW_WORDS;
  b->n_unk++;
  b->raw_n += bytes;
  return 0;
}

/* vmqg_prepare_word_lists over n publishes into pubs / words_out; list
 * elements that are not binaries (VMQGB_NOT_BINARY) become VMQG_WORD_UNKNOWN */
static int prepare_lists(vmqg_ctx* ctx, size_t n, const uint32_t* mountpoints, const uint32_t* counts,
                         const uint8_t* const* words, const size_t* lens, size_t nw, vmqg_pub* pubs,
                         uint32_t* words_out) {
  size_t stack_l[256] = {0};
  size_t* l = nw <= 256 ? stack_l : (size_t*)malloc(nw * sizeof(size_t));
  if (!l) return VMQG_E_NOMEM;
  int nonbin = 0;
  for (size_t k = 0; k < nw; k++) {
    l[k] = lens[k] == VMQGB_NOT_BINARY ? 0 : lens[k];
    nonbin |= lens[k] == VMQGB_NOT_BINARY;
  }
  size_t got = 0;
  const int rc = vmqg_prepare_word_lists(ctx, n, mountpoints, counts, words, l, pubs, words_out, nw, &got);
  if (l != stack_l) free(l);
  if (rc) return rc;
  if (nonbin) {
    for (size_t i = 0; i < n; i++)
      for (uint32_t j = 0; j < pubs[i].nwords; j++)
        if (lens[pubs[i].word_off + j] == VMQGB_NOT_BINARY) {
          words_out[pubs[i].word_off + j] = VMQG_WORD_UNKNOWN;
          pubs[i].flags |= VMQG_PUB_UNKNOWN;
        }
  }
  return 0;
}

int vmqgb_batch_add_word_lists(vmqgb_batch* b, vmqg_ctx* ctx, size_t n, const uint32_t* mountpoints,
                               const uint32_t* counts, const uint8_t* const* words, const size_t* lens,
                               long* idx_out) {
  if (!n) return 0;
  if (b->n == 0) b->dict_gen = vmqg_dict_generation(ctx);
  size_t nw = 0;
  for (size_t i = 0; i < n; i++) nw += counts[i];
  if (grow((void**)&b->pubs, &b->cap, b->n + n, sizeof(vmqg_pub))) return VMQG_E_NOMEM;
  if (grow((void**)&b->words, &b->wcap, b->nwords + nw + 1, sizeof(uint32_t))) return VMQG_E_NOMEM;
  vmqg_pub* P = b->pubs + b->n;
  int rc = prepare_lists(ctx, n, mountpoints, counts, words, lens, nw, P, b->words + b->nwords);
  if (rc) return rc;
  const size_t n_unk0 = b->n_unk, raw0 = b->raw_n;
  for (size_t i = 0; i < n && !rc; i++) {
    const uint32_t off = P[i].word_off;
    if (P[i].flags & VMQG_PUB_UNKNOWN) rc = note_unknown_words(b, b->n + i, P[i].nwords, words + off, lens + off);
    P[i].word_off = off + (uint32_t)b->nwords;
    idx_out[i] = (long)(b->n + i);
  }
  if (rc) { b->n_unk = n_unk0; b->raw_n = raw0; return rc; }
  b->n += n;
  b->nwords += nw;
  return 0;
}

int vmqgb_batch_recheck(vmqgb_batch* b, vmqg_ctx* ctx) {
  if (!b->n_unk) return 0;
  const uint64_t gen = vmqg_dict_generation(ctx);
  if (gen == b->dict_gen) return 0;
  int changed = 0;
  uint32_t tmp[64];
  for (size_t u = 0; u < b->n_unk; u++) {
    vmqg_pub* pub = &b->pubs[b->unk[3 * u]];
    const uint8_t* t = b->raw + b->unk[3 * u + 1];
    const uint32_t rl = b->unk[3 * u + 2];
    const size_t len = rl & ~VMQGB_RAW_WORDS;
    uint32_t* w = pub->nwords <= 64 ? tmp : (uint32_t*)malloc(pub->nwords * sizeof(uint32_t));
    if (!w) return VMQG_E_NOMEM;
    vmqg_pub np;
    int rc;
    if (rl & VMQGB_RAW_WORDS) {   /* a word list: decode its {len, bytes} words */
      const uint32_t c = pub->nwords;
      const uint8_t** wp = (const uint8_t**)malloc((c ? c : 1) * sizeof(*wp));
      size_t* wl = (size_t*)malloc((c ? c : 1) * sizeof(size_t));
      rc = wp && wl ? 0 : VMQG_E_NOMEM;
      const uint8_t* q = t;
      for (uint32_t j = 0; !rc && j < c; j++) {
        uint32_t l;
        memcpy(&l, q, 4);
        q += 4;
        wp[j] = q;
        wl[j] = l == 0xFFFFFFFFu ? VMQGB_NOT_BINARY : l;
        if (l != 0xFFFFFFFFu) q += l;
      }
      if (!rc) rc = prepare_lists(ctx, 1, &pub->mountpoint, &c, wp, wl, c, &np, w);
      free(wp);
      free(wl);
    } else {
      rc = vmqg_prepare_publish(ctx, pub->mountpoint, t, len, w, pub->nwords, &np);
    }
    if (!rc && np.nwords == pub->nwords && memcmp(w, b->words + pub->word_off, np.nwords * sizeof(uint32_t))) {
      memcpy(b->words + pub->word_off, w, np.nwords * sizeof(uint32_t));
      pub->flags = np.flags;
      changed = 1;
    }
    if (w != tmp) free(w);
    if (rc) return rc;
  }
  b->dict_gen = gen;
  return changed;
}

int vmqgb_batch_append(vmqgb_batch* dst, const vmqgb_batch* src) {
  if (grow((void**)&dst->pubs, &dst->cap, dst->n + src->n, sizeof(vmqg_pub))) return VMQG_E_NOMEM;
  if (grow((void**)&dst->words, &dst->wcap, dst->nwords + src->nwords, sizeof(uint32_t))) return VMQG_E_NOMEM;
  if (dst->n == 0 || (src->n && src->dict_gen < dst->dict_gen)) dst->dict_gen = src->dict_gen;
  for (size_t u = 0; u < src->n_unk; u++) {
    const uint32_t* e = src->unk + 3 * u;
    if (note_unknown(dst, dst->n + e[0], src->raw + e[1], e[2])) return VMQG_E_NOMEM;
  }
  memcpy(dst->words + dst->nwords, src->words, src->nwords * sizeof(uint32_t));
  for (size_t i = 0; i < src->n; i++) {
    vmqg_pub p = src->pubs[i];
    p.word_off += (uint32_t)dst->nwords;
    dst->pubs[dst->n + i] = p;
  }
  dst->n += src->n;
  dst->nwords += src->nwords;
  return 0;
}

static int ensure_offsets(vmqgb_batch* b) {   /* n + 1 owned entries */
  if (grow((void**)&b->offs_buf, &b->offs_cap, b->n + 1, sizeof(uint64_t))) return VMQG_E_NOMEM;
  b->offsets = b->offs_buf;
  return 0;
}

int vmqgb_match(vmqgb_batch* b, vmqg_ctx* ctx) {
  if (ensure_offsets(b)) return VMQG_E_NOMEM;
  if (!b->out_cap && grow((void**)&b->out, &b->out_cap, b->n * 4 + 64, sizeof(vmqg_emit))) return VMQG_E_NOMEM;
  if (vmqg_epoch(ctx, &b->epoch)) return VMQG_E_INVAL;
  for (;;) {
    size_t need = 0;
    const int rc = vmqg_match_batch(ctx, b->pubs, b->n, b->words, b->nwords, b->out, b->out_cap, &need, b->offsets);
    if (rc == VMQG_E_OVERFLOW && need > b->out_cap) {   /* grow to the reported total and match again */
      if (grow((void**)&b->out, &b->out_cap, need, sizeof(vmqg_emit))) return VMQG_E_NOMEM;
      continue;
    }
    if (rc) return rc;
    b->out_n = need;
    return 0;
  }
}

int vmqgb_match_ranges(vmqgb_batch* b, vmqg_ctx* ctx) {
  if (ensure_offsets(b)) return VMQG_E_NOMEM;
  if (vmqg_epoch(ctx, &b->epoch)) return VMQG_E_INVAL;
  if (!b->rng_cap && grow((void**)&b->rng_buf, &b->rng_cap, b->n * 2 + 64, sizeof(vmqg_range))) return VMQG_E_NOMEM;
  b->rng = b->rng_buf;
  for (;;) {
    size_t need = 0;
    const int rc = vmqg_match_ranges(ctx, b->pubs, b->n, b->words, b->nwords, b->rng, b->rng_cap, &need, b->offsets);
    if (rc == VMQG_E_OVERFLOW && need > b->rng_cap) {
      if (grow((void**)&b->rng_buf, &b->rng_cap, need, sizeof(vmqg_range))) return VMQG_E_NOMEM;
      b->rng = b->rng_buf;
      continue;
    }
    if (rc) return rc;
    b->rng_n = need;
    return 0;
  }
}

/* ------------------------------------------------------------------ fold */
static vmqgb_entry entry_of(const vmqg_emit* r) {
  vmqgb_entry e;
  e.kind = r->kind_node >> 24;
  e.node = r->kind_node & 0xFFFFFFu;
  e.group = r->group;
  e.subscriber = r->subscriber;
  e.subinfo = r->subinfo;
  return e;
}

size_t vmqgb_count_of(const vmqgb_batch* b, size_t i) {
  return i < b->n ? (size_t)(b->offsets[i + 1] - b->offsets[i]) : 0;
}

int vmqgb_fold(const vmqgb_batch* b, size_t i, vmqgb_fold_fn fn, void* acc) {
  if (i >= b->n) return VMQG_E_INVAL;
  for (uint64_t k = b->offsets[i]; k < b->offsets[i + 1]; k++) {
    const vmqgb_entry e = entry_of(&b->out[k]);
    const int r = fn(acc, &e);
    if (r) return r;
  }
  return 0;
}

int vmqgb_fold_ranges(const vmqgb_batch* b, const vmqg_emit* recs, uint64_t nrecs, size_t i, vmqgb_fold_fn fn,
                      void* acc) {
  if (i >= b->n) return VMQG_E_INVAL;
  for (uint64_t k = b->offsets[i]; k < b->offsets[i + 1]; k++) {
    const vmqg_range g = b->rng[k];
    if (g.count == 0) {   /* remote node: FoldFun(Node, ...) (vmq_reg_trie.erl:78-84) */
      vmqgb_entry e = {VMQG_EMIT_REMOTE, g.off, VMQG_NONE, VMQG_NONE, VMQG_NONE};
      const int r = fn(acc, &e);
      if (r) return r;
      continue;
    }
    if ((uint64_t)g.off + g.count > nrecs) return VMQG_E_STATE;   /* table changed under the ranges */
    for (uint32_t j = 0; j < g.count; j++) {
      const vmqgb_entry e = entry_of(&recs[g.off + j]);
      const int r = fn(acc, &e);
      if (r) return r;
    }
  }
  return 0;
}

int vmqgb_fold_spans(const vmqgb_batch* b, int ranges, const vmqg_emit* recs, uint64_t nrecs, size_t i,
                     vmqgb_span_fn fn, void* acc) {
  if (i >= b->n) return VMQG_E_INVAL;
  if (!ranges) {
    const uint64_t lo = b->offsets[i], hi = b->offsets[i + 1];
    return hi > lo ? fn(acc, b->out + lo, (size_t)(hi - lo)) : 0;
  }
  for (uint64_t k = b->offsets[i]; k < b->offsets[i + 1]; k++) {
    const vmqg_range g = b->rng[k];
    int r;
    if (g.count == 0) {   /* remote node (vmq_reg_trie.erl:78-84) */
      const vmqg_emit e = {(VMQG_EMIT_REMOTE << 24) | g.off, VMQG_NONE, VMQG_NONE, VMQG_NONE};
      r = fn(acc, &e, 1);
    } else {
      if ((uint64_t)g.off + g.count > nrecs) return VMQG_E_STATE;   /* table changed under the ranges */
      r = fn(acc, recs + g.off, g.count);
    }
    if (r) return r;
  }
  return 0;
}

void vmqgb_prefetch_entries(const vmqgb_batch* b, int ranges, const vmqg_emit* recs, uint64_t nrecs, size_t i) {
  if (!ranges || i >= b->n) return;
  for (uint64_t k = b->offsets[i]; k < b->offsets[i + 1]; k++) {
    const vmqg_range g = b->rng[k];
    if (g.count && g.off < nrecs) __builtin_prefetch(recs + g.off);
  }
}

/* ------------------------------------------------------------------- ops */
int vmqgb_ops_init(vmqgb_ops* o) {
  memset(o, 0, sizeof(*o));
  return 0;
}

void vmqgb_ops_reset(vmqgb_ops* o) { o->n = o->nwords = 0; }

void vmqgb_ops_free(vmqgb_ops* o) {
  free(o->ops); free(o->words);
  memset(o, 0, sizeof(*o));
}

int vmqgb_ops_add(vmqgb_ops* o, vmqg_ctx* ctx, uint32_t kind, uint32_t mountpoint, const uint8_t* const* words,
                  const size_t* lens, uint32_t nwords, uint32_t node, uint32_t sub, uint32_t subinfo) {
  if (nwords == 0) return VMQG_E_INVAL;
  if (grow((void**)&o->ops, &o->cap, o->n + 1, sizeof(vmqg_op))) return VMQG_E_NOMEM;
  if (grow((void**)&o->words, &o->wcap, o->nwords + nwords, sizeof(uint32_t))) return VMQG_E_NOMEM;
  /* one blob + offsets for vmqg_intern_words */
  size_t total = 0;
  for (uint32_t i = 0; i < nwords; i++) total += lens[i];
  uint8_t* blob = (uint8_t*)malloc(total ? total : 1);
  uint64_t* offs = (uint64_t*)malloc((nwords + 1) * sizeof(uint64_t));
  if (!blob || !offs) { free(blob); free(offs); return VMQG_E_NOMEM; }
  offs[0] = 0;
  for (uint32_t i = 0; i < nwords; i++) {
    if (lens[i]) memcpy(blob + offs[i], words[i], lens[i]);
    offs[i + 1] = offs[i] + lens[i];
  }
  const int rc = vmqg_intern_words(ctx, blob, offs, nwords, 1, o->words + o->nwords);
  free(blob);
  free(offs);
  if (rc) return rc;
  vmqg_op* op = &o->ops[o->n++];
  op->kind = kind;
  op->mountpoint = mountpoint;
  op->word_off = (uint32_t)o->nwords;
  op->nwords = nwords;
  op->node = node;
  op->subscriber = sub;
  op->subinfo = subinfo;
  op->reserved = 0;
  o->nwords += nwords;
  return 0;
}

int vmqgb_ops_add_filter(vmqgb_ops* o, vmqg_ctx* ctx, uint32_t kind, uint32_t mountpoint, const uint8_t* filter,
                         size_t len, uint32_t node, uint32_t sub, uint32_t subinfo) {
  /* vmq_topic:word splitting keeps empty words ("a//b", "/a") */
  uint32_t n = 1;
  for (size_t i = 0; i < len; i++) n += filter[i] == '/';
  const uint8_t** w = (const uint8_t**)malloc(n * sizeof(*w));
  size_t* l = (size_t*)malloc(n * sizeof(size_t));
  if (!w || !l) { free(w); free(l); return VMQG_E_NOMEM; }
  size_t start = 0;
  uint32_t k = 0;
  for (size_t i = 0; i <= len; i++) {
    if (i == len || filter[i] == '/') { w[k] = filter + start; l[k] = i - start; k++; start = i + 1; }
  }
  const int rc = vmqgb_ops_add(o, ctx, kind, mountpoint, w, l, n, node, sub, subinfo);
  free(w);
  free(l);
  return rc;
}

int vmqgb_ops_apply(vmqgb_ops* o, vmqg_ctx* ctx, uint64_t* epoch) {
  const int rc = vmqg_apply_ops(ctx, o->ops, o->n, o->words, o->nwords, epoch);
  if (rc == 0) vmqgb_ops_reset(o);
  return rc;
}

/* ------------------------------------------------------------------ view */
/* One combined device call in flight (or folded from): the batches it
 * serves, its pinned buffers (vmqg_hbatch) and its results. */
typedef struct vmqgb_req vmqgb_req;
struct vmqgb_req {
  vmqgb_batch* b;
  int dev_ranges;            /* device mode wanted: 1 ranges, 0 records */
  int done, rc;
  size_t base;               /* first publish of the batch in its round */
  struct vmqgb_round* round;
  struct vmqgb_lane* lane;   /* the context its rounds run on */
  vmqgb_req* next;
};

typedef struct vmqgb_round {
  vmqg_hbatch* hb;
  int busy;                  /* taken by a combiner, or leased by batches still reading it */
  int refs;
  int dev_ranges;
  const uint64_t* offs;      /* results (pinned, the hbatch's) */
  const void* out;
  uint64_t epoch;
} vmqgb_round;

/* One device context of the view: lane 0 the primary (host engine + its
 * device tables), lanes 1.. replicas that follow it (vmqg_replica_follow
 * after every commit).  Each lane has its own device mutex, queue and
 * rounds, so the lanes' device calls run side by side. */
typedef struct vmqgb_lane {
  vmqg_ctx* ctx;
  pthread_mutex_t device;    /* the context's device side (submits, commits, follows) */
  vmqgb_req* q_head;         /* under the view's q_mu */
  vmqgb_req* q_tail;
  int in_kernels;            /* rounds submitted whose offsets are not back */
  int ok;                    /* a replica holding a committed epoch of the primary (atomic) */
  int idx;
  vmqgb_round rounds[VMQGB_ROUNDS];
} vmqgb_lane;

/* deferred writer work (vmqgb_view_defer) */
typedef struct vmqgb_deferred {
  void (*fn)(void* arg, uint64_t u);
  void* arg;
  uint64_t u;
  struct vmqgb_deferred* next;
} vmqgb_deferred;

struct vmqgb_view {
  vmqg_ctx* ctx;             /* the primary: dictionary, host engine, readers' record tables */
  /* grace periods: readers are batches between vmqgb_view_enter and
   * vmqgb_view_release, counted per era parity; deferred work waits for a
   * commit that shipped its stage to every lane (pending -> armed), then
   * for the era to flip and the older era's readers to leave (flipped) */
  unsigned era;              /* atomic */
  long readers[2];           /* atomic */
  vmqgb_deferred *pending, *armed, *flipped;   /* the writer's (writer mutex) */
  unsigned flipped_era;
  uint64_t deferred_runs;
  void (*stage_hook)(void* arg, vmqgb_view* v);
  void* stage_hook_arg;
  pthread_mutex_t wr;        /* writers: interning, applies (batchers never take it) */
  pthread_mutex_t q_mu;      /* the queues, the rounds, the counters */
  pthread_cond_t q_cv;
  int inflight;              /* rounds in the kernels per lane, at most */
  int pipelined;             /* the context has a device: hbatch rounds */
  int force_pin_state;       /* tests: the next n range pins answer VMQG_E_STATE */
  int device_records;
  int nlanes;
  unsigned next_lane;        /* vmqgb_view_bind: round robin */
  vmqgb_lane lanes[VMQGB_MAX_LANES];
  vmqgb_view_stats st;
};

static int lane_init(vmqgb_lane* l, vmqg_ctx* ctx, int idx) {
  memset(l, 0, sizeof(*l));
  l->ctx = ctx;
  l->idx = idx;
  if (pthread_mutex_init(&l->device, NULL)) return 0;
  int all = 1;
  for (int i = 0; i < VMQGB_ROUNDS; i++) {
    l->rounds[i].hb = vmqg_hbatch_new(ctx);   /* NULL on a host-engine-only context */
    if (!l->rounds[i].hb) all = 0;
  }
  return all ? 1 : -1;
}

static void lane_free(vmqgb_lane* l) {
  for (int i = 0; i < VMQGB_ROUNDS; i++) vmqg_hbatch_free(l->rounds[i].hb);
  pthread_mutex_destroy(&l->device);
}

vmqgb_view* vmqgb_view_new(vmqg_ctx* ctx) {
  vmqgb_view* v = (vmqgb_view*)calloc(1, sizeof(*v));
  if (!v) return NULL;
  v->ctx = ctx;
  const int r1 = pthread_mutex_init(&v->wr, NULL);
  const int r3 = pthread_mutex_init(&v->q_mu, NULL);
  const int r4 = pthread_cond_init(&v->q_cv, NULL);
  const int r2 = lane_init(&v->lanes[0], ctx, 0);
  if (r1 || r3 || r4 || !r2) { free(v); return NULL; }
  v->nlanes = 1;
  v->lanes[0].ok = 1;
  v->pipelined = r2 == 1;
  v->inflight = 2;
  /* the readers' record buffers: records-mode expansion and range folds read
   * them while the writer stages the next apply */
  if (v->pipelined && vmqg_set_option(ctx, "reader_records", 1) != VMQG_OK) v->pipelined = 0;
  return v;
}

int vmqgb_view_add_replica(vmqgb_view* v, vmqg_ctx* replica) {
  if (!v->pipelined || !replica) return VMQG_E_STATE;
  if (v->nlanes >= VMQGB_MAX_LANES) return VMQG_E_LIMIT;
  vmqgb_lane* l = &v->lanes[v->nlanes];
  if (lane_init(l, replica, v->nlanes) != 1) { lane_free(l); return VMQG_E_NOMEM; }
  vmqgb_view_write_begin(v);
  pthread_mutex_lock(&l->device);
  const int rc = vmqg_replica_follow(replica, v->ctx);   /* the primary's tables as committed now */
  pthread_mutex_unlock(&l->device);
  vmqgb_view_write_end(v);
  if (rc) { lane_free(l); return rc; }
  __atomic_store_n(&l->ok, 1, __ATOMIC_RELEASE);
  pthread_mutex_lock(&v->q_mu);
  v->nlanes++;
  pthread_mutex_unlock(&v->q_mu);
  return 0;
}

int vmqgb_view_lanes(vmqgb_view* v) { return v->nlanes; }

void vmqgb_view_bind(vmqgb_view* v, vmqgb_batch* b) {
  b->lane = __atomic_fetch_add(&v->next_lane, 1u, __ATOMIC_RELAXED) % (unsigned)v->nlanes;
}

static void arm_pending(vmqgb_view* v);
static void run_list(vmqgb_view* v, vmqgb_deferred* d);

void vmqgb_view_free(vmqgb_view* v) {
  if (!v) return;
  /* no reader is left: every deferred free runs now (and what they defer) */
  for (;;) {
    arm_pending(v);
    vmqgb_deferred* d = v->flipped;
    v->flipped = NULL;
    if (!d) { d = v->armed; v->armed = NULL; }
    if (!d) break;
    run_list(v, d);
  }
  for (int k = 0; k < v->nlanes; k++) lane_free(&v->lanes[k]);
  pthread_mutex_destroy(&v->wr);
  pthread_mutex_destroy(&v->q_mu);
  pthread_cond_destroy(&v->q_cv);
  free(v);
}

vmqg_ctx* vmqgb_view_ctx(vmqgb_view* v) { return v->ctx; }

/* ------------------------------------------------------- grace periods */
void vmqgb_view_enter(vmqgb_view* v, vmqgb_batch* b) {
  if (b->in_reader) return;
  for (;;) {
    const unsigned e = __atomic_load_n(&v->era, __ATOMIC_SEQ_CST);
    __atomic_fetch_add(&v->readers[e & 1], 1, __ATOMIC_SEQ_CST);
    if (__atomic_load_n(&v->era, __ATOMIC_SEQ_CST) == e) { b->reader_era = e; b->in_reader = 1; return; }
    __atomic_fetch_sub(&v->readers[e & 1], 1, __ATOMIC_SEQ_CST);   /* flipped meanwhile: count in the new era */
  }
}

static void reader_exit(vmqgb_view* v, vmqgb_batch* b) {
  if (!b->in_reader) return;
  __atomic_fetch_sub(&v->readers[b->reader_era & 1], 1, __ATOMIC_SEQ_CST);
  b->in_reader = 0;
}

int vmqgb_view_defer(vmqgb_view* v, void (*fn)(void*, uint64_t), void* arg, uint64_t u, int after_commit) {
  vmqgb_deferred* d = (vmqgb_deferred*)malloc(sizeof(*d));
  if (!d) return VMQG_E_NOMEM;
  d->fn = fn; d->arg = arg; d->u = u;
  vmqgb_deferred** l = after_commit ? &v->pending : &v->armed;
  d->next = *l;
  *l = d;
  return 0;
}

static void run_list(vmqgb_view* v, vmqgb_deferred* d) {
  while (d) {
    vmqgb_deferred* n = d->next;
    d->fn(d->arg, d->u);
    free(d);
    v->deferred_runs++;
    d = n;
  }
}

/* the writer: runs what the readers have let go of, flips the era for what
 * is armed (writer mutex held) */
void vmqgb_view_reclaim(vmqgb_view* v) {
  for (int round = 0; round < 2; round++) {
    if (v->flipped) {
      if (__atomic_load_n(&v->readers[v->flipped_era & 1], __ATOMIC_SEQ_CST) != 0) return;
      vmqgb_deferred* d = v->flipped;
      v->flipped = NULL;
      run_list(v, d);
    }
    if (!v->armed) return;
    v->flipped = v->armed;
    v->armed = NULL;
    v->flipped_era = __atomic_load_n(&v->era, __ATOMIC_SEQ_CST);
    __atomic_store_n(&v->era, v->flipped_era + 1, __ATOMIC_SEQ_CST);
  }
}

static void arm_pending(vmqgb_view* v) {
  while (v->pending) {
    vmqgb_deferred* d = v->pending;
    v->pending = d->next;
    d->next = v->armed;
    v->armed = d;
  }
}

void vmqgb_view_set_stage_hook(vmqgb_view* v, void (*fn)(void*, vmqgb_view*), void* arg) {
  v->stage_hook = fn;
  v->stage_hook_arg = arg;
}

/* the dictionary's retired words: released after a grace period */
static void dict_release_fn(void* arg, uint64_t token) { vmqg_dict_release((vmqg_ctx*)arg, token); }

/* after a commit (writer mutex held): if every lane holds the committed
 * tables, the stages' deferred work is armed, the words the stages retired
 * are queued for release, and due work runs */
static void after_commit(vmqgb_view* v, int ok) {
  for (int k = 1; ok && k < v->nlanes; k++) ok = __atomic_load_n(&v->lanes[k].ok, __ATOMIC_ACQUIRE);
  if (ok) {
    arm_pending(v);
    vmqgb_view_defer(v, dict_release_fn, v->ctx, vmqg_dict_grace_token(v->ctx), 0);
  }
  vmqgb_view_reclaim(v);
}

void vmqgb_view_grace_stats(vmqgb_view* v, uint64_t* runs, int* waiting) {
  if (runs) *runs = v->deferred_runs;
  if (waiting) *waiting = (v->pending != NULL) + (v->armed != NULL) + (v->flipped != NULL);
}

/* After the primary's commit (writer mutex held): every replica brought to
 * its tables.  A replica that fails keeps answering nothing (its batchers go
 * to the primary) until a later follow succeeds. */
static void follow_replicas(vmqgb_view* v) {
  for (int k = 1; k < v->nlanes; k++) {
    vmqgb_lane* l = &v->lanes[k];
    const uint64_t t0 = mono_ns();
    pthread_mutex_lock(&l->device);
    const int rc = vmqg_replica_follow(l->ctx, v->ctx);
    pthread_mutex_unlock(&l->device);
    const uint64_t t1 = mono_ns();
    __atomic_store_n(&l->ok, rc == 0, __ATOMIC_RELEASE);
    pthread_mutex_lock(&v->q_mu);
    v->st.follow_ns += t1 - t0;
    if (rc) v->st.follow_failures++;
    pthread_mutex_unlock(&v->q_mu);
  }
}

int vmqgb_view_digests(vmqgb_view* v, uint64_t* out, int n) {
  int rc = 0;
  for (int k = 0; k < v->nlanes && k < n && !rc; k++) {
    pthread_mutex_lock(&v->lanes[k].device);
    rc = vmqg_arena_digest(v->lanes[k].ctx, &out[k]);
    pthread_mutex_unlock(&v->lanes[k].device);
  }
  return rc;
}
void vmqgb_view_write_begin(vmqgb_view* v) { pthread_mutex_lock(&v->wr); }
void vmqgb_view_write_end(vmqgb_view* v) { pthread_mutex_unlock(&v->wr); }

/* The host half runs beside the rounds in flight and the batchers' prepares
 * and folds (vmqg_apply_stage reads and writes only the host state and the
 * readers' record buffer nobody is pinned on); the upload takes a turn at
 * the device (the device mutex, after the writer mutex: a device-mutex
 * holder never waits for the writer mutex, so no cycle).  Rounds already
 * submitted stay on the epoch they were submitted at (stream order).  The
 * ops are consumed either way. */
int vmqgb_view_apply_ops(vmqgb_view* v, vmqgb_ops* o, uint64_t* epoch) {
  __atomic_thread_fence(__ATOMIC_RELEASE);   /* the caller's term tables before the ids reach any result */
  const uint64_t t0 = mono_ns();
  int rc = o->n ? vmqg_apply_stage(v->ctx, o->ops, o->n, o->words, o->nwords) : VMQG_OK;
  if (rc == VMQG_E_INVAL || rc == VMQG_E_LIMIT || rc == VMQG_E_STATE) {   /* rejected: nothing staged */
    o->n = o->nwords = 0;
    return rc;
  }
  /* a failed commit leaves the stage pending (the library's contract): the
   * changes are kept and go out with the next commit, whatever its trigger */
  const uint64_t t1 = mono_ns();
  pthread_mutex_lock(&v->lanes[0].device);
  const uint64_t t2 = mono_ns();
  const int rc2 = vmqg_apply_commit(v->ctx, epoch);
  pthread_mutex_unlock(&v->lanes[0].device);
  const uint64_t t3 = mono_ns();
  if (!rc2 && v->nlanes > 1) follow_replicas(v);
  o->n = o->nwords = 0;
  if (!rc && v->stage_hook) v->stage_hook(v->stage_hook_arg, v);   /* the stage's released ids (pending) */
  after_commit(v, rc2 == 0);
  pthread_mutex_lock(&v->q_mu);
  v->st.applies++;
  v->st.stage_ns += t1 - t0;
  v->st.dev_wait_ns += t2 - t1;
  v->st.commit_ns += t3 - t2;
  if (t1 - t0 > v->st.stage_max_ns) v->st.stage_max_ns = t1 - t0;
  if (t2 - t1 > v->st.dev_wait_max_ns) v->st.dev_wait_max_ns = t2 - t1;
  if (t3 - t2 > v->st.commit_max_ns) v->st.commit_max_ns = t3 - t2;
  pthread_mutex_unlock(&v->q_mu);
  return rc ? rc : rc2;
}

int vmqgb_view_commit(vmqgb_view* v, uint64_t* epoch) {
  vmqgb_view_write_begin(v);
  pthread_mutex_lock(&v->lanes[0].device);
  const int rc = vmqg_apply_commit(v->ctx, epoch);
  pthread_mutex_unlock(&v->lanes[0].device);
  if (!rc && v->nlanes > 1) follow_replicas(v);
  after_commit(v, rc == 0);
  vmqgb_view_write_end(v);
  return rc;
}

int vmqgb_view_set_option(vmqgb_view* v, const char* name, int64_t value) {
  if (strcmp(name, "force_pin_state") == 0) {   /* the batch layer's own (tests: the ranges fallback) */
    if (value < 0 || value > (1 << 30)) return VMQG_E_INVAL;
    __atomic_store_n(&v->force_pin_state, (int)value, __ATOMIC_RELAXED);
    return 0;
  }
  vmqgb_view_write_begin(v);
  pthread_mutex_lock(&v->lanes[0].device);
  const int rc = vmqg_set_option(v->ctx, name, value);
  pthread_mutex_unlock(&v->lanes[0].device);
  /* kernel knobs on the replicas too (the primary-only ones they refuse) */
  for (int k = 1; !rc && k < v->nlanes; k++) {
    pthread_mutex_lock(&v->lanes[k].device);
    vmqg_set_option(v->lanes[k].ctx, name, value);
    pthread_mutex_unlock(&v->lanes[k].device);
  }
  vmqgb_view_write_end(v);
  return rc;
}

int vmqgb_view_ctx_stats(vmqgb_view* v, vmqg_stats_t* out) {
  /* the writer's fields under the writer mutex, the device calls' (epoch,
   * arena size, last-call counters) under the device mutex: the order an
   * apply takes them in */
  vmqgb_view_write_begin(v);
  pthread_mutex_lock(&v->lanes[0].device);
  const int rc = vmqg_stats(v->ctx, out);
  pthread_mutex_unlock(&v->lanes[0].device);
  vmqgb_view_write_end(v);
  return rc;
}

int vmqgb_view_apply(vmqgb_view* v, vmqgb_ops* o, uint64_t* epoch) {
  vmqgb_view_write_begin(v);
  const int rc = vmqgb_view_apply_ops(v, o, epoch);
  vmqgb_view_write_end(v);
  return rc;
}

void vmqgb_view_set_device_records(vmqgb_view* v, int on) { v->device_records = on != 0; }
void vmqgb_view_set_inflight(vmqgb_view* v, int n) {
  pthread_mutex_lock(&v->q_mu);
  v->inflight = n < 1 ? 1 : n > VMQGB_ROUNDS - 1 ? VMQGB_ROUNDS - 1 : n;
  pthread_cond_broadcast(&v->q_cv);
  pthread_mutex_unlock(&v->q_mu);
}

void vmqgb_view_get_stats(vmqgb_view* v, vmqgb_view_stats* out) {
  pthread_mutex_lock(&v->q_mu);
  *out = v->st;
  pthread_mutex_unlock(&v->q_mu);
}

void vmqgb_view_reset_stats(vmqgb_view* v) {
  pthread_mutex_lock(&v->q_mu);
  memset(&v->st, 0, sizeof v->st);
  pthread_mutex_unlock(&v->q_mu);
}

static void round_release(vmqgb_view* v, vmqgb_round* r) {   /* q_mu held */
  if (--r->refs == 0) {
    r->busy = 0;
    pthread_cond_broadcast(&v->q_cv);
  }
}

/* the batch's pinned record table and round buffers (its reader section goes on) */
static void release_lease(vmqgb_view* v, vmqgb_batch* b);

void vmqgb_view_release(vmqgb_view* v, vmqgb_batch* b) {
  release_lease(v, b);
  reader_exit(v, b);
}

static void release_lease(vmqgb_view* v, vmqgb_batch* b) {
  if (b->rec_pinned) {
    vmqg_records_unpin(v->ctx, b->rec_pin);
    b->rec_pinned = 0;
  }
  if (!b->lease) return;
  pthread_mutex_lock(&v->q_mu);
  round_release(v, (vmqgb_round*)b->lease);
  pthread_mutex_unlock(&v->q_mu);
  b->lease = NULL;
  b->offsets = b->offs_buf;
  b->rng = b->rng_buf;
}

/* A combiner's round: the taken batches' publishes and words concatenated
 * into the hbatch's pinned inputs, one submit under the device mutex, the
 * offsets (the next round may start then), the entries, the hand-out. */
static void run_round(vmqgb_view* v, vmqgb_lane* lane, vmqgb_round* r, vmqgb_req* list) {
  size_t n = 0, nw = 0;
  for (vmqgb_req* q = list; q; q = q->next) { q->base = n; n += q->b->n; nw += q->b->nwords; }
  vmqg_pub* P = NULL;
  uint32_t* W = NULL;
  int rc = vmqg_hbatch_inputs(r->hb, n, nw, &P, &W);
  if (!rc) {
    size_t wb = 0;
    for (vmqgb_req* q = list; q; q = q->next) {
      const vmqgb_batch* b = q->b;
      memcpy(W + wb, b->words, b->nwords * sizeof(uint32_t));
      vmqg_pub* d = P + q->base;
      for (size_t i = 0; i < b->n; i++) {
        d[i] = b->pubs[i];
        d[i].word_off += (uint32_t)wb;
      }
      wb += b->nwords;
    }
  }
  const uint64_t* offs = NULL;
  uint64_t total = 0, epoch = 0;
  for (int attempt = 0; !rc; attempt++) {
    pthread_mutex_lock(&lane->device);
    rc = vmqg_hbatch_submit(lane->ctx, r->hb, n, nw, r->dev_ranges);
    pthread_mutex_unlock(&lane->device);
    if (rc) break;
    rc = vmqg_hbatch_offsets(r->hb, &offs, &total, &epoch);
    if ((rc == VMQG_E_OVERFLOW || rc == VMQG_E_FRONTIER) && attempt < 8) {   /* larger output / stack: again */
      pthread_mutex_lock(&v->q_mu);
      v->st.overflow_retries++;
      pthread_mutex_unlock(&v->q_mu);
      rc = 0;
      continue;
    }
    break;
  }
  pthread_mutex_lock(&v->q_mu);
  lane->in_kernels--;
  pthread_cond_broadcast(&v->q_cv);
  pthread_mutex_unlock(&v->q_mu);
  const void* out = NULL;
  if (!rc) rc = vmqg_hbatch_entries(r->hb, &out);
  r->offs = offs;
  r->out = out;
  r->epoch = epoch;
  pthread_mutex_lock(&v->q_mu);
  v->st.rounds++;
  v->st.lane_rounds[lane->idx]++;
  v->st.round_publishes += n;
  if (n > v->st.max_round_publishes) v->st.max_round_publishes = n;
  r->refs = 0;
  for (vmqgb_req* q = list; q; q = q->next) {
    v->st.round_batches++;
    q->rc = rc;
    q->round = rc ? NULL : r;
    if (!rc) r->refs++;
    q->done = 1;
  }
  if (r->refs == 0) r->busy = 0;
  pthread_cond_broadcast(&v->q_cv);
  pthread_mutex_unlock(&v->q_mu);
}

/* Queues req and returns when a round has served it (q_mu not held on entry
 * or exit).  A waiting batcher becomes the combiner when fewer than
 * v->inflight rounds are in the kernels and a round is free: it takes the
 * queued batches of the head's device mode, up to VMQGB_ROUND_MAX publishes. */
static void combine(vmqgb_view* v, vmqgb_req* req) {
  vmqgb_lane* lane = req->lane;
  pthread_mutex_lock(&v->q_mu);
  req->done = 0;
  req->next = NULL;
  if (lane->q_tail) lane->q_tail->next = req; else lane->q_head = req;
  lane->q_tail = req;
  while (!req->done) {
    vmqgb_round* r = NULL;
    if (lane->q_head && lane->in_kernels < v->inflight)
      for (int i = 0; i < VMQGB_ROUNDS && !r; i++) if (!lane->rounds[i].busy) r = &lane->rounds[i];
    if (!r) { pthread_cond_wait(&v->q_cv, &v->q_mu); continue; }
    /* take the head's mode, FIFO, up to the round's publish budget */
    const int mode = lane->q_head->dev_ranges;
    vmqgb_req *list = NULL, *tail = NULL, **pp = &lane->q_head, *last = NULL;
    size_t n = 0;
    while (*pp) {
      vmqgb_req* q = *pp;
      if (q->dev_ranges == mode && (n == 0 || n + q->b->n <= VMQGB_ROUND_MAX)) {
        *pp = q->next;
        q->next = NULL;
        if (tail) tail->next = q; else list = q;
        tail = q;
        n += q->b->n;
      } else {
        last = q;
        pp = &q->next;
      }
    }
    lane->q_tail = last;
    r->busy = 1;
    r->dev_ranges = mode;
    lane->in_kernels++;
    pthread_mutex_unlock(&v->q_mu);
    run_round(v, lane, r, list);
    pthread_mutex_lock(&v->q_mu);
  }
  pthread_mutex_unlock(&v->q_mu);
}

/* records mode: the batch's records copied out of its round (device
 * records) or expanded from the readers' record table of the round's epoch
 * (device ranges, pinned for the copy); offsets rebased to the batch. */
static int expand_ranges(vmqgb_batch* b, const uint64_t* o, const vmqg_range* g, const vmqg_emit* recs,
                         uint64_t nrecs);
static int take_records(vmqgb_view* v, vmqgb_batch* b, vmqgb_req* q) {
  const vmqgb_round* r = q->round;
  const uint64_t* o = r->offs + q->base;
  if (ensure_offsets(b)) return VMQG_E_NOMEM;
  if (!r->dev_ranges) {
    const uint64_t first = o[0], cnt = o[b->n] - first;
    if (grow((void**)&b->out, &b->out_cap, cnt + 1, sizeof(vmqg_emit))) return VMQG_E_NOMEM;
    memcpy(b->out, (const vmqg_emit*)r->out + first, cnt * sizeof(vmqg_emit));
    for (size_t i = 0; i <= b->n; i++) b->offsets[i] = o[i] - first;
    b->out_n = cnt;
    return 0;
  }
  const vmqg_range* g = (const vmqg_range*)r->out;
  uint64_t cnt = 0;
  for (uint64_t k = o[0]; k < o[b->n]; k++) cnt += g[k].count ? g[k].count : 1;
  if (grow((void**)&b->out, &b->out_cap, cnt + 1, sizeof(vmqg_emit))) return VMQG_E_NOMEM;
  const vmqg_emit* recs = NULL;
  uint64_t nrecs = 0;
  uint32_t pin = 0;
  int rc = vmqg_records_pin(v->ctx, r->epoch, &recs, &nrecs, &pin);
  if (rc) return rc;   /* VMQG_E_STATE: two applies rewrote record slots since the round */
  rc = expand_ranges(b, o, g, recs, nrecs);
  vmqg_records_unpin(v->ctx, pin);
  return rc;
}

static int expand_ranges(vmqgb_batch* b, const uint64_t* o, const vmqg_range* g, const vmqg_emit* recs,
                         uint64_t nrecs) {
  vmqg_emit* dst = b->out;
  b->offsets[0] = 0;
  for (size_t i = 0; i < b->n; i++) {
    for (uint64_t k = o[i]; k < o[i + 1]; k++) {
      const vmqg_range e = g[k];
      if (e.count == 0) {   /* remote node (fold_/5, vmq_reg_trie.erl:78-84) */
        dst->kind_node = (VMQG_EMIT_REMOTE << 24) | e.off;
        dst->group = dst->subscriber = dst->subinfo = VMQG_NONE;
        dst++;
        continue;
      }
      if ((uint64_t)e.off + e.count > nrecs) return VMQG_E_STATE;
      memcpy(dst, recs + e.off, (size_t)e.count * sizeof(vmqg_emit));
      dst += e.count;
    }
    b->offsets[i + 1] = (uint64_t)(dst - b->out);
  }
  b->out_n = b->offsets[b->n];
  return 0;
}

/* without a device (host-engine contexts): one synchronous call, which
 * reports VMQG_E_DEVICE */
static int match_records(vmqgb_view* v, vmqgb_batch* b, vmqgb_req* qp, int dev_ranges);

static int match_direct(vmqgb_view* v, vmqgb_batch* b, int ranges, const vmqg_emit** recs, uint64_t* nrecs) {
  (void)recs; (void)nrecs;
  pthread_mutex_lock(&v->lanes[0].device);
  const int rc = ranges ? vmqgb_match_ranges(b, v->ctx) : vmqgb_match(b, v->ctx);
  pthread_mutex_unlock(&v->lanes[0].device);
  return rc ? rc : VMQG_E_DEVICE;
}

int vmqgb_view_match(vmqgb_view* v, vmqgb_batch* b, int ranges, const vmqg_emit** recs, uint64_t* nrecs) {
  release_lease(v, b);
  vmqgb_view_enter(v, b);   /* no-op when the batch entered before its prepare */
  b->out_ranges = ranges;
  if (recs) *recs = NULL;
  if (nrecs) *nrecs = 0;
  if (b->n == 0) {   /* nothing to match: empty results */
    if (ensure_offsets(b)) return VMQG_E_NOMEM;
    b->offsets[0] = 0;
    b->out_n = b->rng_n = 0;
    return 0;
  }
  if (!v->pipelined) return match_direct(v, b, ranges, recs, nrecs);
  vmqgb_req q;
  memset(&q, 0, sizeof q);
  q.b = b;
  /* the batch's lane, unless that replica is not following (then the primary's) */
  {
    const unsigned k = b->lane < (unsigned)v->nlanes ? b->lane : 0u;
    q.lane = &v->lanes[k && __atomic_load_n(&v->lanes[k].ok, __ATOMIC_ACQUIRE) ? k : 0];
  }
  if (ranges) {
    /* the round's entries stay in its buffers and the record table of its
     * epoch stays pinned until the caller has folded (vmqgb_view_release) */
    for (int attempt = 0;; attempt++) {
      q.dev_ranges = 1;
      combine(v, &q);
      if (q.rc) return q.rc;
      const vmqgb_round* r = q.round;
      b->lease = q.round;
      b->offsets = (uint64_t*)(r->offs + q.base);
      b->rng = (vmqg_range*)r->out;
      b->rng_n = r->offs[q.base + b->n] - r->offs[q.base];
      b->epoch = r->epoch;
      const vmqg_emit* rt = NULL;
      uint64_t nrt = 0;
      int rc = vmqg_records_pin(v->ctx, b->epoch, &rt, &nrt, &b->rec_pin);
      if (rc == 0) b->rec_pinned = 1;
      if (rc == 0 && __atomic_load_n(&v->force_pin_state, __ATOMIC_RELAXED) > 0 &&
          __atomic_sub_fetch(&v->force_pin_state, 1, __ATOMIC_RELAXED) >= 0)
        rc = VMQG_E_STATE;   /* as if two applies had rewritten the record slots (release_lease unpins) */
      if (rc == VMQG_E_STATE) {   /* two applies rewrote record slots since the round */
        release_lease(v, b);
        pthread_mutex_lock(&v->q_mu);
        v->st.state_retries++;
        pthread_mutex_unlock(&v->q_mu);
        if (attempt < 3) continue;
        /* applies keep outrunning the rounds: this batch takes the records
         * path with device-copied records (no pin needed), as records mode
         * does; the caller folds b->out (b->out_ranges == 0) */
        b->out_ranges = 0;
        pthread_mutex_lock(&v->q_mu);
        v->st.ranges_fallbacks++;
        pthread_mutex_unlock(&v->q_mu);
        return match_records(v, b, &q, 0);
      }
      if (rc) return rc;
      rc = vmqgb_batch_recheck(b, v->ctx);   /* a word became known after the prepare */
      if (rc < 0) return rc;
      if (rc == 1 && attempt < 16) {
        b->stale_rematches++;
        release_lease(v, b);
        pthread_mutex_lock(&v->q_mu);
        v->st.stale_rematches++;
        pthread_mutex_unlock(&v->q_mu);
        continue;
      }
      if (recs) *recs = rt;
      if (nrecs) *nrecs = nrt;
      return 0;
    }
  }
  /* records: the records are copied out of the round (the expansion pins
   * the record table of the round's epoch for the copy only) */
  return match_records(v, b, &q, !v->device_records);
}

static int match_records(vmqgb_view* v, vmqgb_batch* b, vmqgb_req* qp, int dev_ranges) {
  vmqgb_req q = *qp;
  for (int attempt = 0;; attempt++) {
    q.dev_ranges = dev_ranges;
    combine(v, &q);
    if (q.rc) return q.rc;
    int rc = take_records(v, b, &q);
    b->epoch = q.round->epoch;
    pthread_mutex_lock(&v->q_mu);
    round_release(v, q.round);
    if (!rc) { if (dev_ranges) v->st.expanded_batches++; else v->st.device_record_batches++; }
    if (rc == VMQG_E_STATE) v->st.state_retries++;
    pthread_mutex_unlock(&v->q_mu);
    if (rc == VMQG_E_STATE && dev_ranges) { dev_ranges = 0; continue; }   /* the device copies the records */
    if (rc) return rc;
    /* a word unknown at prepare time may have subscriptions on the tables
     * this batch was matched on: prepare those publishes again and match */
    rc = vmqgb_batch_recheck(b, v->ctx);
    if (rc < 0) return rc;
    if (rc == 1 && attempt < 16) {
      b->stale_rematches++;
      pthread_mutex_lock(&v->q_mu);
      v->st.stale_rematches++;
      pthread_mutex_unlock(&v->q_mu);
      continue;
    }
    return 0;
  }
}
