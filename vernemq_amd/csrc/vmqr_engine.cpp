// Retained store host engine (see vmqr_engine.h).  Citations are to
// apps/vmq_server/src/vmq_retain_srv.erl unless noted.
#include "vmqr_engine.h"
#include "vmqg_chain.h"

#include <algorithm>
#include <cstring>

namespace vmqr {

using vmqg::kEmpty;
using vmqg::kNone;

static uint64_t next_pow2(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}
static uint64_t align256(uint64_t v) { return (v + 255) & ~255ull; }

RetainEngine::~RetainEngine() {
  if (!has_device) return;
  hipSetDevice(device);
  if (stream) hipStreamSynchronize(stream);
  for (auto* v : {&t_count, &t_scan, &t_emit})
    for (auto& e : *v) { hipEventDestroy(e.first); hipEventDestroy(e.second); }
  if (ev_match_done) hipEventDestroy(ev_match_done);
  hipFree(d_arena); hipFree(d_patch); hipFree(d_status); hipFree(d_tickets); hipFree(d_plan); hipFree(d_lookback);
  hipFree(d_f); hipFree(d_w); hipFree(d_o); hipFree(d_offs);
  if (h_patch) hipHostFree(h_patch);
  if (stream) hipStreamDestroy(stream);
}

int RetainEngine::init(const vmqr_config& c) {
  cfg = c;
  if (cfg.max_mountpoints == 0) cfg.max_mountpoints = 1024;
  if (cfg.max_mountpoints > vmqg::kMaxMountpoints) return VMQG_E_LIMIT;
  for (const char* s : {"+", "#", "$share"}) intern(reinterpret_cast<const uint8_t*>(s), strlen(s), true);
  mplists.resize(cfg.max_mountpoints);
  rebuild();
  if (cfg.device >= 0) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || cfg.device >= n) return VMQG_E_DEVICE;
    device = cfg.device;
    if (hipSetDevice(device) != hipSuccess) return VMQG_E_DEVICE;
    if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return VMQG_E_DEVICE;
    if (hipEventCreateWithFlags(&ev_match_done, hipEventDisableTiming) != hipSuccess) return VMQG_E_DEVICE;
    has_device = true;
    if (hipMalloc(&d_status, 64) != hipSuccess) return VMQG_E_NOMEM;
    if (hipMalloc(&d_tickets, 8 * kTicketStride * 4) != hipSuccess) return VMQG_E_NOMEM;
    if (hipDeviceGetAttribute(&cu_count, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cu_count < 1)
      cu_count = 256;
    // the walk's grid is what fits on the chip at once (every block resident)
    walk_grid = std::max(8, cu_count * walk_blocks_per_cu());
    return upload();
  }
  return VMQG_OK;
}

uint32_t RetainEngine::intern(const uint8_t* b, size_t n, bool create) {
  std::string s(reinterpret_cast<const char*>(b), n);
  auto it = word_index.find(s);
  if (it != word_index.end()) return it->second;
  if (!create) return vmqg::kUnknownWord;
  const uint32_t id = (uint32_t)word_text.size();
  word_text.push_back(s);
  word_index.emplace(std::move(s), id);
  return id;
}

// ------------------------------------------------------------------ mirror
void RetainEngine::touch(uint64_t off, uint64_t bytes) {
  if (full_image) return;
  for (uint64_t c = off >> 4, e = (off + bytes + 15) >> 4; c < e; c++) {
    uint64_t& w = dirty_bits[c >> 6];
    const uint64_t bit = 1ull << (c & 63);
    if (!(w & bit)) { w |= bit; dirty_chunks.push_back(c); }
  }
}

RLayout RetainEngine::plan_layout(uint32_t scale) const {
  RLayout L{};
  L.magic = kRLayoutMagic;
  L.max_mp = cfg.max_mountpoints;
  uint64_t words = 0, lists = 0;
  for (auto& r : rows) words += r.words.size();
  for (auto& p : parts) lists += std::max<uint64_t>(4, next_pow2(p.rows.size()));
  for (auto& m : mplists) if (!m.rows.empty()) lists += std::max<uint64_t>(4, next_pow2(m.rows.size()));
  L.rows_cap = std::max<uint64_t>({4096, rows.size() * 2, cfg.hint_topics}) * scale;
  L.rwords_cap = std::max<uint64_t>(16384, words * 2 + cfg.hint_topics * 8) * scale;
  L.lists_cap = std::max<uint64_t>(16384, lists * 2 + cfg.hint_topics * 8) * scale;
  // slot load <= 1/8 after a re-layout, <= 1/4 before the next (place_part)
  L.ptab_buckets = next_pow2(std::max<uint64_t>({1024, parts.size() * 4, cfg.hint_topics})) * scale;
  L.exact_slots = next_pow2(std::max<uint64_t>({4096, rows.size() * 2 + 1024, cfg.hint_topics * 2})) * scale;
  uint64_t o = 0;
  L.rows_off = o;   o = align256(o + L.rows_cap * sizeof(RRow));
  L.rwords_off = o; o = align256(o + L.rwords_cap * 4);
  L.lists_off = o;  o = align256(o + L.lists_cap * sizeof(LEnt));
  L.ptab_off = o;   o = align256(o + L.ptab_buckets * kPSlotsPerBucket * sizeof(PSlot));
  L.mpl_off = o;    o = align256(o + L.max_mp * sizeof(MpList));
  L.exact_off = o;  o = align256(o + L.exact_slots * sizeof(XSlot));
  L.total_bytes = o;
  return L;
}

// Re-lay the arena out from the logical state (lists packed, exact table
// without tombstones); the next upload ships the whole image.
void RetainEngine::rebuild() {
  for (uint32_t scale = 1;; scale *= 2) {
    lay = plan_layout(scale);
    mirror.assign(lay.total_bytes / 8, 0);
    memset(region<uint8_t>(lay.ptab_off), 0xFF, lay.ptab_buckets * kPSlotsPerBucket * sizeof(PSlot));
    dirty_bits.assign((lay.total_bytes / 16 + 63) / 64, 0);
    dirty_chunks.clear();
    full_image = true;
    rwords_top = lists_top = lists_garbage = exact_used = 0;
    bool ok = true;
    for (auto& r : rows) { r.words_off = kNone; r.xslot = ~0ull; }
    for (uint32_t r = 0; ok && r < rows.size(); r++) ok = write_row(r) && (!rows[r].live || place_exact(r));
    auto lay_list = [&](RList& l) {
      l.cap = std::max<uint64_t>(4, next_pow2(l.rows.size()));
      if (lists_top + l.cap > lay.lists_cap) return false;
      l.off = lists_top; lists_top += l.cap;
      LEnt* pool = region<LEnt>(lay.lists_off) + l.off;
      for (size_t i = 0; i < l.rows.size(); i++) pool[i] = entry_of(l.rows[i]);
      return true;
    };
    for (uint32_t p = 0; ok && p < parts.size(); p++) {
      part_slot[p] = ~0ull;
      ok = lay_list(parts[p]) && place_part(p);
    }
    for (uint32_t m = 0; ok && m < mplists.size(); m++) {
      RList& l = mplists[m];
      if (l.rows.empty()) { l.off = 0; l.cap = 0; continue; }
      ok = lay_list(l) && write_list_head(false, m);
    }
    if (ok) break;
  }
  rebuilds++;
}

bool RetainEngine::write_row(uint32_t r) {
  RRowInfo& R = rows[r];
  if (r >= lay.rows_cap) return false;
  if (R.words_off == kNone) {
    if (rwords_top + R.words.size() > lay.rwords_cap) return false;
    R.words_off = (uint32_t)rwords_top;
    std::copy(R.words.begin(), R.words.end(), region<uint32_t>(lay.rwords_off) + rwords_top);
    touch(lay.rwords_off + rwords_top * 4, R.words.size() * 4);
    rwords_top += R.words.size();
  }
  *(region<RRow>(lay.rows_off) + r) = RRow{R.msg, (uint32_t)R.words.size(), R.words_off, R.mp};
  touch(lay.rows_off + (uint64_t)r * sizeof(RRow), sizeof(RRow));
  return true;
}

LEnt RetainEngine::entry_of(uint32_t r) const {
  const RRowInfo& R = rows[r];
  LEnt e{r, R.msg, (uint32_t)R.words.size(), R.words_off, {0, 0, 0, 0}};
  for (uint32_t k = 0; k < kLWords && k < R.words.size(); k++) e.w[k] = R.words[k];
  return e;
}

void RetainEngine::put_entry(uint64_t slot, uint32_t r) {
  // after a capacity miss in this batch the arena is laid out anew anyway
  if (full_image || slot >= lay.lists_cap) return;
  region<LEnt>(lay.lists_off)[slot] = entry_of(r);
  touch(lay.lists_off + slot * sizeof(LEnt), sizeof(LEnt));
}

// Exact slot of a live row (a revived row reuses its slot; tombstones are
// only cleared by a re-layout).
bool RetainEngine::place_exact(uint32_t r) {
  RRowInfo& R = rows[r];
  XSlot* tab = region<XSlot>(lay.exact_off);
  const uint64_t fp = retain_fp(R.mp, R.words.data(), (uint32_t)R.words.size());
  if (R.xslot == ~0ull) {
    if ((exact_used + 1) * 2 > lay.exact_slots) return false;
    const uint64_t mask = lay.exact_slots - 1;
    uint64_t i = fp & mask;
    while (tab[i].state != 0) i = (i + 1) & mask;
    R.xslot = i;
    exact_used++;
  }
  tab[R.xslot] = XSlot{fp, r, R.live ? kXLive : kXTomb};
  touch(lay.exact_off + R.xslot * sizeof(XSlot), sizeof(XSlot));
  return true;
}

bool RetainEngine::place_part(uint32_t p) {
  if ((uint64_t)(p + 1) * 4 > lay.ptab_buckets * kPSlotsPerBucket) return false;   // keep the load <= 1/4
  PSlot* tab = region<PSlot>(lay.ptab_off);
  const uint64_t mask = lay.ptab_buckets - 1;
  for (uint64_t b = part_hash(part_mp[p], part_a[p], part_b[p], part_kind[p]) & mask;; b = (b + 1) & mask) {
    for (uint32_t j = 0; j < kPSlotsPerBucket; j++) {
      const uint64_t si = b * kPSlotsPerBucket + j;
      if (tab[si].mp == kEmpty) {
        part_slot[p] = si;
        return write_list_head(true, p);
      }
    }
  }
}

bool RetainEngine::write_list_head(bool part, uint32_t id) {
  if (part) {
    if (part_slot[id] == ~0ull) return false;   // no table slot (capacity): the caller re-lays out
    const RList& l = parts[id];
    PSlot& s = region<PSlot>(lay.ptab_off)[part_slot[id]];
    s = PSlot{part_mp[id], part_a[id], part_b[id], part_kind[id], (uint32_t)l.off, (uint32_t)l.rows.size(), {0, 0}};
    touch(lay.ptab_off + part_slot[id] * sizeof(PSlot), sizeof(PSlot));
  } else {
    const RList& l = mplists[id];
    region<MpList>(lay.mpl_off)[id] = MpList{(uint32_t)l.off, (uint32_t)l.rows.size()};
    touch(lay.mpl_off + (uint64_t)id * sizeof(MpList), sizeof(MpList));
  }
  return true;
}

// Append `row` to one of its lists (relocating the list when it is full);
// returns false when the list pool is exhausted (the caller re-lays the
// arena out).
bool RetainEngine::list_push(uint32_t row, int which) {
  RRowInfo& R = rows[row];
  const bool part = which >= 0;
  const uint32_t id = part ? R.part[which] : R.mp;
  RList& l = part ? parts[id] : mplists[id];
  const uint32_t pos = (uint32_t)l.rows.size();
  (part ? R.ppos[which] : R.mpos) = pos;
  l.rows.push_back(row);
  if (l.rows.size() > l.cap) {
    const uint64_t cap = std::max<uint64_t>(4, next_pow2(l.rows.size()));
    if (lists_top + cap > lay.lists_cap) return false;
    lists_garbage += l.cap;
    l.off = lists_top; l.cap = cap; lists_top += cap;
    for (size_t i = 0; i < l.rows.size(); i++) put_entry(l.off + i, l.rows[i]);
  } else {
    put_entry(l.off + pos, row);
  }
  return write_list_head(part, id);
}

// Swap-remove of `row` from one of its lists (order inside a list is free:
// ets:foldl order is unspecified).  The row moved into the hole finds its
// own slot for the list by the list id (a row is in a list at most once).
void RetainEngine::list_remove(uint32_t row, int which) {
  RRowInfo& R = rows[row];
  const bool part = which >= 0;
  const uint32_t id = part ? R.part[which] : R.mp;
  RList& l = part ? parts[id] : mplists[id];
  uint32_t& mine = part ? R.ppos[which] : R.mpos;
  const uint32_t pos = mine;
  const uint32_t last = l.rows.back();
  l.rows.pop_back();
  if (pos < l.rows.size()) {
    l.rows[pos] = last;
    RRowInfo& M = rows[last];
    if (part) {
      for (size_t j = 0; j < M.part.size(); j++) if (M.part[j] == id) { M.ppos[j] = pos; break; }
    } else {
      M.mpos = pos;
    }
    put_entry(l.off + pos, last);
  }
  mine = kNone;
  write_list_head(part, id);
}

uint32_t RetainEngine::find_row(uint32_t mp, const uint32_t* w, uint32_t L) const {
  return key_index.find(retain_fp(mp, w, L), [&](uint32_t r) {
    const RRowInfo& R = rows[r];
    return R.mp == mp && R.words.size() == L && std::equal(R.words.begin(), R.words.end(), w);
  });
}

// The list {MP, kind, a, b}: kPair {MP, w0, w1}, kPos {MP, word, position}.
uint32_t RetainEngine::part_of(uint32_t mp, uint32_t a, uint32_t b, uint32_t kind) {
  const uint64_t h = part_hash(mp, a, b, kind);
  const uint32_t f = part_index.find(h, [&](uint32_t p) {
    return part_mp[p] == mp && part_a[p] == a && part_b[p] == b && part_kind[p] == kind;
  });
  if (f != FlatIndex::kVoid) return f;
  const uint32_t p = (uint32_t)parts.size();
  parts.emplace_back();
  part_mp.push_back(mp); part_a.push_back(a); part_b.push_back(b); part_kind.push_back(kind);
  part_slot.push_back(~0ull);
  part_index.insert(h, p);
  return p;
}

// insert/3 (:68-71): ets:insert into a set — an existing key takes the new value.
void RetainEngine::insert(uint32_t mp, const uint32_t* w, uint32_t L, uint32_t msg) {
  uint32_t r = find_row(mp, w, L);
  bool ok = true;
  if (r != FlatIndex::kVoid && rows[r].live) {
    RRowInfo& R = rows[r];
    R.msg = msg;
    ok = write_row(r);
    // the list entries carry the msg
    for (size_t j = 0; j < R.part.size(); j++) put_entry(parts[R.part[j]].off + R.ppos[j], r);
    put_entry(mplists[R.mp].off + R.mpos, r);
  } else {
    if (r == FlatIndex::kVoid) {
      r = (uint32_t)rows.size();
      rows.emplace_back();
      RRowInfo& N = rows[r];
      N.mp = mp;
      N.words.assign(w, w + L);
      if (L >= 2) N.part.push_back(part_of(mp, w[0], w[1], kPair));
      for (uint32_t k = 0; k < L && k < kMaxPos; k++) N.part.push_back(part_of(mp, w[k], k, kPos));
      N.ppos.assign(N.part.size(), kNone);
      key_index.insert(retain_fp(mp, w, L), r);
    }
    RRowInfo& R = rows[r];
    R.msg = msg;
    R.live = true;
    n_live++;
    ok = write_row(r);   // first: the list entries copy its words offset
    for (size_t j = 0; j < R.part.size(); j++) {
      const uint32_t id = R.part[j];
      if (part_slot[id] == ~0ull) ok = place_part(id) && ok;
      ok = list_push(r, (int)j) && ok;
    }
    ok = list_push(r, -1) && ok;
    ok = ok && place_exact(r);
  }
  if (!ok) full_image = true;   // capacity: apply() re-lays out
}

// delete/2 (:63-66): ets:delete — a missing key is a no-op.
void RetainEngine::erase(uint32_t mp, const uint32_t* w, uint32_t L) {
  const uint32_t r = find_row(mp, w, L);
  if (r == FlatIndex::kVoid || !rows[r].live) return;
  RRowInfo& R = rows[r];
  R.live = false;
  n_live--;
  for (size_t j = 0; j < R.part.size(); j++) list_remove(r, (int)j);
  list_remove(r, -1);
  if (R.xslot != ~0ull) place_exact(r);   // tombstone
}

int RetainEngine::apply(const vmqr_op* ops, size_t n, const uint32_t* words, size_t nwords) {
  uint32_t top_mp = 0;
  for (size_t i = 0; i < n; i++) {   // validate the whole batch first
    const vmqr_op& o = ops[i];
    if (o.kind != VMQR_OP_INSERT && o.kind != VMQR_OP_DELETE) return VMQG_E_INVAL;
    if (o.mountpoint >= vmqg::kMaxMountpoints) return VMQG_E_LIMIT;
    if (o.mountpoint >= top_mp) top_mp = o.mountpoint + 1;
    if (o.nwords == 0 || (uint64_t)o.word_off + o.nwords > nwords) return VMQG_E_INVAL;
    for (uint32_t j = 0; j < o.nwords; j++) if (words[o.word_off + j] >= word_text.size()) return VMQG_E_INVAL;
  }
  // a retained topic on a mountpoint past the per-mountpoint lists grows
  // them (doubling; vmq_retain_srv keys by {MP, Topic} with no limit,
  // vmq_retain_srv.erl:53-66): a re-layout before any op touches the arena
  if (top_mp > cfg.max_mountpoints) {
    uint64_t m = cfg.max_mountpoints;
    while (m < top_mp) m *= 2;
    cfg.max_mountpoints = (uint32_t)std::min<uint64_t>(m, vmqg::kMaxMountpoints);
    mplists.resize(cfg.max_mountpoints);
    rebuild();
  }
  // a capacity miss inside insert/erase sets full_image: the logical state
  // stays exact, touches stop, and the arena is laid out anew below
  const bool grown = full_image;
  full_image = false;
  for (size_t i = 0; i < n; i++) {
    const vmqr_op& o = ops[i];
    if (o.kind == VMQR_OP_INSERT) insert(o.mountpoint, words + o.word_off, o.nwords, o.msg);
    else erase(o.mountpoint, words + o.word_off, o.nwords);
  }
  if (full_image || lists_garbage > lay.lists_cap / 2) rebuild();
  else if (grown) full_image = true;   // the re-layout above: the upload ships the image
  epoch++;
  return upload();
}

int RetainEngine::upload() {
  std::vector<Patch> patches;
  if (!full_image && dirty_chunks.size() * sizeof(Patch) > lay.total_bytes / 2) full_image = true;
  if (!full_image) {
    patches.reserve(dirty_chunks.size());
    const uint8_t* base = reinterpret_cast<const uint8_t*>(mirror.data());
    for (uint64_t c : dirty_chunks) {
      Patch p;
      p.off = c * 16;
      memcpy(p.data, base + p.off, 16);
      patches.push_back(p);
      dirty_bits[c >> 6] = 0;
    }
  } else {
    std::fill(dirty_bits.begin(), dirty_bits.end(), 0);
  }
  dirty_chunks.clear();
  if (!has_device) { full_image = false; return VMQG_OK; }
  hipSetDevice(device);
  // tables must not change under a match still reading them
  if (order_on(stream) != VMQG_OK) return VMQG_E_DEVICE;
  if (full_image) {
    if (hipStreamSynchronize(stream) != hipSuccess) return VMQG_E_DEVICE;
    if (d_arena_bytes < lay.total_bytes) {
      if (d_arena) hipFree(d_arena);
      d_arena = nullptr; d_arena_bytes = 0;
      if (hipMalloc(&d_arena, lay.total_bytes) != hipSuccess) return VMQG_E_NOMEM;
      d_arena_bytes = lay.total_bytes;
    }
    if (hipMemcpyAsync(d_arena, mirror.data(), lay.total_bytes, hipMemcpyHostToDevice, stream) != hipSuccess)
      return VMQG_E_DEVICE;
    if (hipStreamSynchronize(stream) != hipSuccess) return VMQG_E_DEVICE;
    full_image = false;
    return VMQG_OK;
  }
  const uint64_t np = patches.size();
  if (np == 0) return VMQG_OK;
  if (h_patch_cap < np) {
    if (h_patch) hipHostFree(h_patch);
    h_patch = nullptr;
    h_patch_cap = next_pow2(np);
    if (hipHostMalloc(&h_patch, h_patch_cap * sizeof(Patch)) != hipSuccess) { h_patch_cap = 0; return VMQG_E_NOMEM; }
  }
  if (d_patch_cap < np) {
    if (d_patch) hipFree(d_patch);
    d_patch = nullptr;
    d_patch_cap = next_pow2(np);
    if (hipMalloc(&d_patch, d_patch_cap * sizeof(Patch)) != hipSuccess) { d_patch_cap = 0; return VMQG_E_NOMEM; }
  }
  memcpy(h_patch, patches.data(), np * sizeof(Patch));
  if (hipMemcpyAsync(d_patch, h_patch, np * sizeof(Patch), hipMemcpyHostToDevice, stream) != hipSuccess)
    return VMQG_E_DEVICE;
  if (vmqg::launch_patches(d_arena, d_patch, np, stream) != hipSuccess) return VMQG_E_DEVICE;
  if (hipStreamSynchronize(stream) != hipSuccess) return VMQG_E_DEVICE;
  return VMQG_OK;
}

// -------------------------------------------------------------- matching
int RetainEngine::match_device(const vmqg_pub* d_filters, uint32_t nf, const uint32_t* d_words, uint32_t* d_out,
                               uint64_t out_cap, uint64_t* d_offsets, hipStream_t st) {
  if (!has_device) return VMQG_E_DEVICE;
  hipSetDevice(device);
  // match_fold must not read tables a pending patch upload is writing: the
  // context's stream is synchronised at the end of every apply; later
  // applies wait for this match (order_on).  The status words and the walk
  // tickets are zeroed by k_rt_plan (no memset launches).
  if (order_on(st) != VMQG_OK) return VMQG_E_DEVICE;
  if (nf == 0) {
    if (hipMemsetAsync(d_status, 0, 32, st) != hipSuccess) return VMQG_E_DEVICE;
    return hipMemsetAsync(d_offsets, 0, 8, st) == hipSuccess ? VMQG_OK : VMQG_E_DEVICE;
  }
  if (nf + 1 > plan_cap) {
    if (d_plan) { hipStreamSynchronize(st); hipFree(d_plan); }
    d_plan = nullptr;
    plan_cap = next_pow2(nf + 1);
    if (hipMalloc(&d_plan, plan_cap * 3 * sizeof(uint64_t)) != hipSuccess) { plan_cap = 0; return VMQG_E_NOMEM; }
  }
  // look-back granules: the filter scan's tiles and the walk's tiles (the
  // walk's row count is only known on the device: a batch needing more
  // reports VMQG_E_FRONTIER and vmqr_match_batch grows and reruns)
  if (int rc = grow_tiles(std::max<uint64_t>(walk_rows_hint, (uint64_t)nf * 64), st)) return rc;
  last_nf = nf;
  lb_tag += 2;   // two look-back passes per call, one tag each
  if (lb_tag + 1 >= (1u << 20)) {
    if (hipMemsetAsync(d_lookback, 0, lookback_cap * 8, st) != hipSuccess) return VMQG_E_DEVICE;
    lb_tag = 2;
  }
  RArgs a{};
  a.rows = reinterpret_cast<const RRow*>(d_arena + lay.rows_off);
  a.rwords = reinterpret_cast<const uint32_t*>(d_arena + lay.rwords_off);
  a.lists = reinterpret_cast<const LEnt*>(d_arena + lay.lists_off);
  a.ptab = reinterpret_cast<const PSlot*>(d_arena + lay.ptab_off);
  a.ptab_mask = lay.ptab_buckets - 1;
  a.mpl = reinterpret_cast<const MpList*>(d_arena + lay.mpl_off);
  a.max_mp = (uint32_t)lay.max_mp;
  a.exact = reinterpret_cast<const XSlot*>(d_arena + lay.exact_off);
  a.exact_mask = lay.exact_slots - 1;
  a.filters = d_filters; a.words = d_words; a.nf = nf;
  a.plan = d_plan; a.rpfx = d_plan + 2 * plan_cap;
  a.out = d_out; a.out_cap = out_cap; a.offsets = d_offsets;
  a.status = d_status; a.lookback = d_lookback; a.lb_tag = lb_tag; a.tile_cap = lookback_cap;
  a.tickets = d_tickets;
  hipEvent_t e[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  if (timing) for (auto& x : e) hipEventCreate(&x);
  if (launch_retain_match(a, (uint32_t)walk_grid, st, timing ? e : nullptr) != hipSuccess) return VMQG_E_DEVICE;
  if (timing) { t_count.push_back({e[0], e[1]}); t_scan.push_back({e[2], e[3]}); t_emit.push_back({e[4], e[5]}); }
  return VMQG_OK;
}

// Patches and matches form one chain across streams (vmqg_chain.h).
int RetainEngine::order_on(hipStream_t st) { return vmqg::chain_order(ev_match_done, ev_stream, st); }

int RetainEngine::grow_tiles(uint64_t rows, hipStream_t st) {
  const uint64_t want = std::max<uint64_t>(rows / kTileRows + 2, (plan_cap + 4095) / 4096 + 2);
  if (want <= lookback_cap) return VMQG_OK;
  if (d_lookback) { hipStreamSynchronize(st); hipFree(d_lookback); }
  d_lookback = nullptr;
  lookback_cap = next_pow2(want);
  if (hipMalloc(&d_lookback, lookback_cap * 8) != hipSuccess) { lookback_cap = 0; return VMQG_E_NOMEM; }
  if (hipMemsetAsync(d_lookback, 0, lookback_cap * 8, st) != hipSuccess) return VMQG_E_DEVICE;
  lb_tag = 2;
  return VMQG_OK;
}

int RetainEngine::match_status(hipStream_t st) {
  if (!has_device) return VMQG_E_DEVICE;
  hipSetDevice(device);
  if (order_on(st) != VMQG_OK) return VMQG_E_DEVICE;
  uint32_t h[8] = {0};
  if (hipMemcpyAsync(h, d_status, 32, hipMemcpyDeviceToHost, st) != hipSuccess) return VMQG_E_DEVICE;
  if (hipStreamSynchronize(st) != hipSuccess) return VMQG_E_DEVICE;
  if (hipMemsetAsync(d_status, 0, 32, st) != hipSuccess) return VMQG_E_DEVICE;
  if (h[1] & 32u) {
    // look-back tiles exhausted: size them from the batch's row count, so
    // that the same batch succeeds when it is run again
    uint64_t need = 0;
    if (hipMemcpy(&need, d_plan + 2 * plan_cap + last_nf, 8, hipMemcpyDeviceToHost) != hipSuccess) return VMQG_E_DEVICE;
    if (int rc = grow_tiles(need, st)) return rc;
    return VMQG_E_FRONTIER;
  }
  if (h[1] & 4u) return VMQG_E_OVERFLOW;
  if (h[1]) return VMQG_E_DEVICE;
  return VMQG_OK;
}

void RetainEngine::collect_times() {
  if (!has_device) return;
  for (size_t i = 0; i < t_count.size(); i++) {
    float a = 0, a2 = 0, b = 0;
    hipEventSynchronize(t_emit[i].second);
    hipEventElapsedTime(&a, t_count[i].first, t_count[i].second);
    hipEventElapsedTime(&a2, t_scan[i].first, t_scan[i].second);
    hipEventElapsedTime(&b, t_emit[i].first, t_emit[i].second);
    sum_count_ns += (a + a2) * 1e6; sum_emit_ns += b * 1e6; n_timed++;
    for (auto* v : {&t_count, &t_scan, &t_emit}) { hipEventDestroy((*v)[i].first); hipEventDestroy((*v)[i].second); }
  }
  t_count.clear(); t_scan.clear(); t_emit.clear();
}

std::string RetainEngine::dump() {
  std::vector<std::string> lines;
  for (const RRowInfo& R : rows) {
    if (!R.live) continue;
    std::string l = "mp#" + std::to_string(R.mp) + " [";
    for (size_t i = 0; i < R.words.size(); i++) {
      if (i) l += ",";
      l += word_text[R.words[i]];
    }
    lines.push_back(l + "] -> msg#" + std::to_string(R.msg));
  }
  std::sort(lines.begin(), lines.end());
  std::string out;
  for (auto& l : lines) { out += l; out += '\n'; }
  return out;
}

}  // namespace vmqr
