/*
 * vmqg_batch.c — see vmqg_batch.h.  Plain C99, no OTP, no HIP: only the
 * libvmqgpu C ABI.
 */
#define _GNU_SOURCE   /* pthread_rwlockattr_setkind_np: writers are not starved by readers */
#include "vmqg_batch.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------ interner */
struct vmqgb_interner {
  uint8_t* bytes;       /* every key, back to back */
  size_t nbytes, bcap;
  uint64_t* offs;       /* id -> start in bytes (offs[id + 1] = end) */
  uint32_t n, ocap;
  uint32_t* slots;      /* open addressing: id + 1, 0 = empty */
  uint64_t* hashes;     /* per slot */
  uint32_t mask;
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
  t->offs = (uint64_t*)calloc(t->ocap + 1, sizeof(uint64_t));
  if (!t->slots || !t->hashes || !t->offs) { vmqgb_interner_free(t); return NULL; }
  return t;
}

void vmqgb_interner_free(vmqgb_interner* t) {
  if (!t) return;
  free(t->bytes); free(t->offs); free(t->slots); free(t->hashes); free(t);
}

static int eq_at(const vmqgb_interner* t, uint32_t id, const void* bytes, size_t len) {
  const uint64_t a = t->offs[id], e = t->offs[id + 1];
  return e - a == len && memcmp(t->bytes + a, bytes, len) == 0;
}

static void rehash(vmqgb_interner* t) {
  const uint32_t ncap = (t->mask + 1) * 2;
  uint32_t* s = (uint32_t*)calloc(ncap, sizeof(uint32_t));
  uint64_t* h = (uint64_t*)calloc(ncap, sizeof(uint64_t));
  if (!s || !h) { free(s); free(h); return; }   /* keeps the old table: still correct, only fuller */
  for (uint32_t i = 0; i <= t->mask; i++) {
    if (!t->slots[i]) continue;
    uint32_t j = (uint32_t)t->hashes[i] & (ncap - 1);
    while (s[j]) j = (j + 1) & (ncap - 1);
    s[j] = t->slots[i];
    h[j] = t->hashes[i];
  }
  free(t->slots); free(t->hashes);
  t->slots = s; t->hashes = h; t->mask = ncap - 1;
}

int vmqgb_lookup(const vmqgb_interner* t, const void* bytes, size_t len, uint32_t* id) {
  const uint64_t hv = hash_bytes(bytes, len);
  for (uint32_t j = (uint32_t)hv & t->mask;; j = (j + 1) & t->mask) {
    const uint32_t v = t->slots[j];
    if (!v) return -1;
    if (t->hashes[j] == hv && eq_at(t, v - 1, bytes, len)) { if (id) *id = v - 1; return 0; }
  }
}

uint32_t vmqgb_intern(vmqgb_interner* t, const void* bytes, size_t len) {
  const uint64_t hv = hash_bytes(bytes, len);
  uint32_t j = (uint32_t)hv & t->mask;
  for (;; j = (j + 1) & t->mask) {
    const uint32_t v = t->slots[j];
    if (!v) break;
    if (t->hashes[j] == hv && eq_at(t, v - 1, bytes, len)) return v - 1;
  }
  if (t->nbytes + len > t->bcap) {
    size_t c = t->bcap ? t->bcap * 2 : 4096;
    while (c < t->nbytes + len) c *= 2;
    uint8_t* nb = (uint8_t*)realloc(t->bytes, c);
    if (!nb) return VMQG_NONE;
    t->bytes = nb; t->bcap = c;
  }
  if (t->n + 1 >= t->ocap) {
    uint64_t* no = (uint64_t*)realloc(t->offs, (size_t)(t->ocap * 2 + 1) * sizeof(uint64_t));
    if (!no) return VMQG_NONE;
    t->offs = no; t->ocap *= 2;
  }
  const uint32_t id = t->n++;
  if (len) memcpy(t->bytes + t->nbytes, bytes, len);
  t->nbytes += len;
  t->offs[id + 1] = t->nbytes;
  t->slots[j] = id + 1;
  t->hashes[j] = hv;
  if ((uint64_t)t->n * 2 > t->mask + 1) rehash(t);
  return id;
}

const uint8_t* vmqgb_bytes(const vmqgb_interner* t, uint32_t id, size_t* len) {
  if (id >= t->n) return NULL;
  if (len) *len = (size_t)(t->offs[id + 1] - t->offs[id]);
  return t->bytes + t->offs[id];
}

uint32_t vmqgb_count(const vmqgb_interner* t) { return t->n; }

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

void vmqgb_batch_reset(vmqgb_batch* b) { b->n = b->nwords = b->out_n = b->rng_n = 0; }

void vmqgb_batch_free(vmqgb_batch* b) {
  free(b->pubs); free(b->words); free(b->offsets); free(b->out); free(b->rng);
  memset(b, 0, sizeof(*b));
}

long vmqgb_batch_add(vmqgb_batch* b, vmqg_ctx* ctx, uint32_t mountpoint, const uint8_t* topic, size_t len) {
  if (grow((void**)&b->pubs, &b->cap, b->n + 1, sizeof(vmqg_pub))) return VMQG_E_NOMEM;
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
    b->nwords += pub.nwords;
    b->pubs[b->n] = pub;
    return (long)b->n++;
  }
}

int vmqgb_batch_append(vmqgb_batch* dst, const vmqgb_batch* src) {
  if (grow((void**)&dst->pubs, &dst->cap, dst->n + src->n, sizeof(vmqg_pub))) return VMQG_E_NOMEM;
  if (grow((void**)&dst->words, &dst->wcap, dst->nwords + src->nwords, sizeof(uint32_t))) return VMQG_E_NOMEM;
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

static int ensure_offsets(vmqgb_batch* b) {   /* n + 1 entries, sized per call */
  void* p = realloc(b->offsets, (b->n + 1) * sizeof(uint64_t));
  if (!p) return VMQG_E_NOMEM;
  b->offsets = (uint64_t*)p;
  return 0;
}

int vmqgb_match(vmqgb_batch* b, vmqg_ctx* ctx) {
  if (ensure_offsets(b)) return VMQG_E_NOMEM;
  if (!b->out_cap && grow((void**)&b->out, &b->out_cap, b->n * 4 + 64, sizeof(vmqg_emit))) return VMQG_E_NOMEM;
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
  if (!b->rng_cap && grow((void**)&b->rng, &b->rng_cap, b->n * 2 + 64, sizeof(vmqg_range))) return VMQG_E_NOMEM;
  for (;;) {
    size_t need = 0;
    const int rc = vmqg_match_ranges(ctx, b->pubs, b->n, b->words, b->nwords, b->rng, b->rng_cap, &need, b->offsets);
    if (rc == VMQG_E_OVERFLOW && need > b->rng_cap) {
      if (grow((void**)&b->rng, &b->rng_cap, need, sizeof(vmqg_range))) return VMQG_E_NOMEM;
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
struct vmqgb_view {
  vmqg_ctx* ctx;
  pthread_rwlock_t tables;   /* readers: batchers; writers: applies */
  pthread_mutex_t device;    /* one device call at a time */
};

vmqgb_view* vmqgb_view_new(vmqg_ctx* ctx) {
  vmqgb_view* v = (vmqgb_view*)calloc(1, sizeof(*v));
  if (!v) return NULL;
  v->ctx = ctx;
  pthread_rwlockattr_t a;
  pthread_rwlockattr_init(&a);
  pthread_rwlockattr_setkind_np(&a, PTHREAD_RWLOCK_PREFER_WRITER_NONRECURSIVE_NP);
  const int r1 = pthread_rwlock_init(&v->tables, &a);
  pthread_rwlockattr_destroy(&a);
  const int r2 = pthread_mutex_init(&v->device, NULL);
  if (r1 || r2) { free(v); return NULL; }
  return v;
}

void vmqgb_view_free(vmqgb_view* v) {
  if (!v) return;
  pthread_rwlock_destroy(&v->tables);
  pthread_mutex_destroy(&v->device);
  free(v);
}

vmqg_ctx* vmqgb_view_ctx(vmqgb_view* v) { return v->ctx; }
void vmqgb_view_read_begin(vmqgb_view* v) { pthread_rwlock_rdlock(&v->tables); }
void vmqgb_view_read_end(vmqgb_view* v) { pthread_rwlock_unlock(&v->tables); }
void vmqgb_view_yield(vmqgb_view* v) {   /* a waiting writer goes first (writer-preferring lock) */
  pthread_rwlock_unlock(&v->tables);
  pthread_rwlock_rdlock(&v->tables);
}
/* A writer takes the device mutex too: a records-mode batch matches without
 * the read lock, and an apply changes what a match reads (the layout, the
 * arena, the staging ring).  Order: the write lock, then the mutex; a mutex
 * holder never waits for the table lock, so no cycle. */
void vmqgb_view_write_begin(vmqgb_view* v) {
  pthread_rwlock_wrlock(&v->tables);
  pthread_mutex_lock(&v->device);
}
void vmqgb_view_write_end(vmqgb_view* v) {
  pthread_mutex_unlock(&v->device);
  pthread_rwlock_unlock(&v->tables);
}

int vmqgb_view_match(vmqgb_view* v, vmqgb_batch* b, int ranges, const vmqg_emit** recs, uint64_t* nrecs) {
  if (b->n == 0) {   /* nothing to match: empty results */
    if (ensure_offsets(b)) return VMQG_E_NOMEM;
    b->offsets[0] = 0;
    b->out_n = b->rng_n = 0;
    if (recs) *recs = NULL;
    if (nrecs) *nrecs = 0;
    return 0;
  }
  /* records are copies: the read lock is let go while the batch waits for
   * the device, so an apply can land between this batch's prepare and its
   * match (its word ids stay valid: the dictionary only grows) and a writer
   * never waits for a queue of device calls.  Ranges index the host record
   * table: they keep the lock until the caller has folded them. */
  if (!ranges) vmqgb_view_read_end(v);
  pthread_mutex_lock(&v->device);
  int rc = ranges ? vmqgb_match_ranges(b, v->ctx) : vmqgb_match(b, v->ctx);
  pthread_mutex_unlock(&v->device);
  if (!ranges) vmqgb_view_read_begin(v);
  if (!rc && ranges && recs && nrecs) rc = vmqg_records_at(v->ctx, b->epoch, recs, nrecs);
  return rc;
}

int vmqgb_view_apply(vmqgb_view* v, vmqgb_ops* o, uint64_t* epoch) {
  vmqgb_view_write_begin(v);
  const int rc = vmqgb_ops_apply(o, v->ctx, epoch);
  vmqgb_view_write_end(v);
  return rc;
}
