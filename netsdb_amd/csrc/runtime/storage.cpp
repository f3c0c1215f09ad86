// Page files, LRU buffer manager and slab allocator (host side of the netsdb_amd storage layer).
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "runtime.h"

namespace nsdb_rt {

// ================================================================== SlabAllocator
SlabAllocator::SlabAllocator(uint64_t capacity, uint64_t alignment) : cap_(capacity), align_(alignment ? alignment : 256) {
  if (capacity) insert_free(0, capacity);
}

void SlabAllocator::insert_free(uint64_t off, uint64_t sz) {
  free_[off] = sz;
  by_size_.emplace(sz, off);
}

void SlabAllocator::erase_free(uint64_t off, uint64_t sz) {
  free_.erase(off);
  auto range = by_size_.equal_range(sz);
  for (auto it = range.first; it != range.second; ++it)
    if (it->second == off) {
      by_size_.erase(it);
      break;
    }
}

int64_t SlabAllocator::alloc(uint64_t bytes) {
  std::lock_guard<std::mutex> g(mu_);
  if (bytes == 0) bytes = 1;
  const uint64_t need = (bytes + align_ - 1) / align_ * align_;
  auto it = by_size_.lower_bound(need);      // best fit
  if (it == by_size_.end()) return -1;
  const uint64_t sz = it->first, off = it->second;
  erase_free(off, sz);
  if (sz > need) insert_free(off + need, sz - need);
  live_[off] = need;
  used_ += need;
  return (int64_t)off;
}

void SlabAllocator::free(int64_t offset) {
  std::lock_guard<std::mutex> g(mu_);
  auto lv = live_.find((uint64_t)offset);
  if (lv == live_.end()) throw std::runtime_error("SlabAllocator::free: unknown offset");
  uint64_t off = lv->first, sz = lv->second;
  live_.erase(lv);
  used_ -= sz;
  // coalesce with neighbours
  auto nxt = free_.lower_bound(off);
  if (nxt != free_.end() && off + sz == nxt->first) {
    uint64_t nsz = nxt->second, noff = nxt->first;
    erase_free(noff, nsz);
    sz += nsz;
  }
  auto prv = free_.lower_bound(off);
  if (prv != free_.begin()) {
    --prv;
    if (prv->first + prv->second == off) {
      uint64_t poff = prv->first, psz = prv->second;
      erase_free(poff, psz);
      off = poff;
      sz += psz;
    }
  }
  insert_free(off, sz);
}

uint64_t SlabAllocator::largest_free() const {
  std::lock_guard<std::mutex> g(mu_);
  return by_size_.empty() ? 0 : by_size_.rbegin()->first;
}

// ================================================================== PageFile
PageFile::PageFile(const std::string& path, uint64_t page_size) : path_(path), page_size_(page_size) {
  fd_ = ::open(path.c_str(), O_RDWR | O_CREAT, 0644);
  if (fd_ < 0) throw std::runtime_error("PageFile: cannot open " + path);
  load_meta();
}

PageFile::~PageFile() {
  if (fd_ >= 0) {
    save_meta();
    ::close(fd_);
  }
}

void PageFile::load_meta() {
  std::ifstream f(path_ + ".meta");
  if (!f) return;
  uint64_t ps, n;
  f >> ps >> n;
  if (ps != page_size_) throw std::runtime_error("PageFile: page size mismatch for " + path_);
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t p, l;
    f >> p >> l;
    lengths_[p] = l;
  }
}

void PageFile::save_meta() {
  std::ofstream f(path_ + ".meta", std::ios::trunc);
  f << page_size_ << " " << lengths_.size() << "\n";
  for (auto& kv : lengths_) f << kv.first << " " << kv.second << "\n";
}

void PageFile::write_page(uint64_t page_no, const void* data, uint64_t bytes) {
  std::lock_guard<std::mutex> g(mu_);
  if (bytes > page_size_) throw std::runtime_error("PageFile::write_page: page overflow");
  const char* p = (const char*)data;
  uint64_t done = 0;
  while (done < bytes) {
    ssize_t w = ::pwrite(fd_, p + done, bytes - done, (off_t)(page_no * page_size_ + done));
    if (w <= 0) throw std::runtime_error("PageFile::write_page: pwrite failed on " + path_);
    done += (uint64_t)w;
  }
  lengths_[page_no] = bytes;
}

uint64_t PageFile::read_page(uint64_t page_no, void* out, uint64_t cap) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = lengths_.find(page_no);
  if (it == lengths_.end()) throw std::runtime_error("PageFile::read_page: no such page");
  const uint64_t n = std::min(it->second, cap);
  char* p = (char*)out;
  uint64_t done = 0;
  while (done < n) {
    ssize_t r = ::pread(fd_, p + done, n - done, (off_t)(page_no * page_size_ + done));
    if (r <= 0) throw std::runtime_error("PageFile::read_page: pread failed on " + path_);
    done += (uint64_t)r;
  }
  return n;
}

bool PageFile::has_page(uint64_t page_no) const {
  std::lock_guard<std::mutex> g(mu_);
  return lengths_.count(page_no) > 0;
}

std::vector<uint64_t> PageFile::pages() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<uint64_t> v;
  for (auto& kv : lengths_) v.push_back(kv.first);
  return v;
}

void PageFile::sync() {
  std::lock_guard<std::mutex> g(mu_);
  save_meta();
  ::fsync(fd_);
}

// ================================================================== BufferManager
BufferManager::BufferManager(uint64_t page_size, uint64_t num_pages, const std::string& spill_dir)
    : page_size_(page_size), num_slots_(num_pages), dir_(spill_dir) {
  if (page_size == 0 || num_pages == 0) throw std::runtime_error("BufferManager: empty pool");
  ::mkdir(dir_.c_str(), 0755);
  if (posix_memalign((void**)&arena_, 4096, page_size * num_pages) != 0)
    throw std::runtime_error("BufferManager: cannot allocate page pool");
  frames_.resize(num_pages);
  for (int64_t i = (int64_t)num_pages - 1; i >= 0; --i) free_slots_.push_back(i);
}

BufferManager::~BufferManager() {
  try {
    flush_all();
  } catch (...) {
  }
  for (auto& kv : files_) delete kv.second;
  std::free(arena_);
}

PageFile* BufferManager::file_for(int64_t set_id) {
  auto it = files_.find(set_id);
  if (it != files_.end()) return it->second;
  auto* f = new PageFile(dir_ + "/set_" + std::to_string(set_id) + ".pages", page_size_);
  files_[set_id] = f;
  for (auto p : f->pages()) known_[set_id].emplace((int64_t)p, 0);
  return f;
}

void BufferManager::write_back(int64_t slot) {
  Frame& fr = frames_[slot];
  if (!fr.dirty) return;
  file_for(fr.key.set_id)->write_page((uint64_t)fr.key.page_no, arena_ + slot * page_size_, fr.used);
  fr.dirty = false;
}

int64_t BufferManager::grab_slot() {
  if (!free_slots_.empty()) {
    int64_t s = free_slots_.back();
    free_slots_.pop_back();
    return s;
  }
  if (lru_.empty()) throw std::runtime_error("BufferManager: all pages pinned (pool exhausted)");
  int64_t victim = lru_.front();
  lru_.pop_front();
  Frame& fr = frames_[victim];
  fr.in_lru = false;
  write_back(victim);
  table_.erase(fr.key);
  fr.key = {-1, -1};
  ++evictions_;
  return victim;
}

int64_t BufferManager::pin(int64_t set_id, int64_t page_no, bool create) {
  std::lock_guard<std::mutex> g(mu_);
  PageKey k{set_id, page_no};
  auto it = table_.find(k);
  if (it != table_.end()) {
    Frame& fr = frames_[it->second];
    if (fr.in_lru) {
      lru_.erase(fr.lru_it);
      fr.in_lru = false;
    }
    ++fr.pins;
    return it->second;
  }
  PageFile* f = file_for(set_id);
  const bool on_disk = f->has_page((uint64_t)page_no);
  if (!on_disk && !create) throw std::runtime_error("BufferManager::pin: page does not exist");
  int64_t slot = grab_slot();
  Frame& fr = frames_[slot];
  fr.key = k;
  fr.pins = 1;
  fr.dirty = false;
  fr.used = 0;
  if (on_disk) {
    fr.used = f->read_page((uint64_t)page_no, arena_ + slot * page_size_, page_size_);
    ++loads_;
  } else {
    fr.dirty = true;   // a new page must reach the file when evicted
  }
  table_[k] = slot;
  known_[set_id][page_no] = fr.used;
  return slot;
}

void BufferManager::unpin(int64_t set_id, int64_t page_no, bool dirty, uint64_t bytes_used) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = table_.find(PageKey{set_id, page_no});
  if (it == table_.end()) throw std::runtime_error("BufferManager::unpin: page not resident");
  Frame& fr = frames_[it->second];
  if (fr.pins <= 0) throw std::runtime_error("BufferManager::unpin: page not pinned");
  if (dirty) {
    fr.dirty = true;
    fr.used = std::min(bytes_used, page_size_);
    known_[set_id][page_no] = fr.used;
  }
  if (--fr.pins == 0) {
    lru_.push_back(it->second);
    fr.lru_it = std::prev(lru_.end());
    fr.in_lru = true;
  }
}

bool BufferManager::drop_page(int64_t set_id, int64_t page_no) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = table_.find(PageKey{set_id, page_no});
  if (it != table_.end()) {
    Frame& fr = frames_[it->second];
    if (fr.pins > 0) return false;
    if (fr.in_lru) lru_.erase(fr.lru_it);
    fr = Frame();
    free_slots_.push_back(it->second);
    table_.erase(it);
  }
  auto k = known_.find(set_id);
  if (k != known_.end()) k->second.erase(page_no);
  return true;
}

void BufferManager::drop_set(int64_t set_id) {
  std::lock_guard<std::mutex> g(mu_);
  for (auto it = table_.begin(); it != table_.end();) {
    if (it->first.set_id == set_id) {
      Frame& fr = frames_[it->second];
      if (fr.in_lru) lru_.erase(fr.lru_it);
      fr = Frame();
      free_slots_.push_back(it->second);
      it = table_.erase(it);
    } else {
      ++it;
    }
  }
  auto f = files_.find(set_id);
  std::string path = dir_ + "/set_" + std::to_string(set_id) + ".pages";
  if (f != files_.end()) {
    path = f->second->path();
    delete f->second;
    files_.erase(f);
  }
  ::unlink(path.c_str());
  ::unlink((path + ".meta").c_str());
  known_.erase(set_id);
}

void BufferManager::flush_set(int64_t set_id) {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& kv : table_)
    if (kv.first.set_id == set_id) write_back(kv.second);
  if (files_.count(set_id)) files_[set_id]->sync();
}

bool BufferManager::prefetch(int64_t set_id, int64_t page_no) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (table_.count(PageKey{set_id, page_no})) return false;       // already resident
    PageFile* f = file_for(set_id);
    if (!f->has_page((uint64_t)page_no)) return false;
  }
  pin(set_id, page_no, false);
  unpin(set_id, page_no, false, 0);
  return true;
}

void BufferManager::flush_all() {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& kv : table_) write_back(kv.second);
  for (auto& kv : files_) kv.second->sync();
}

uint8_t* BufferManager::slot_ptr(int64_t slot) {
  if (slot < 0 || (uint64_t)slot >= num_slots_) throw std::runtime_error("BufferManager: bad slot");
  return arena_ + slot * page_size_;
}

uint64_t BufferManager::bytes_used(int64_t set_id, int64_t page_no) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = known_.find(set_id);
  if (it == known_.end()) return 0;
  auto p = it->second.find(page_no);
  return p == it->second.end() ? 0 : p->second;
}

int64_t BufferManager::resident_pages() const {
  std::lock_guard<std::mutex> g(mu_);
  return (int64_t)table_.size();
}

std::vector<int64_t> BufferManager::set_pages(int64_t set_id) const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<int64_t> v;
  auto it = known_.find(set_id);
  if (it != known_.end())
    for (auto& kv : it->second) v.push_back(kv.first);
  return v;
}

// ================================================================== hashing
uint64_t hash64(uint64_t x) {   // splitmix64 finaliser
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

void hash_columns(const int64_t* const* cols, int ncols, int64_t n, uint64_t* out) {
  for (int64_t i = 0; i < n; ++i) {
    uint64_t h = 0x84222325CBF29CE4ull;
    for (int c = 0; c < ncols; ++c) h = hash64(h ^ (uint64_t)cols[c][i]);
    out[i] = h;
  }
}

void partition_ids(const uint64_t* hashes, int64_t n, int nparts, int32_t* out) {
  for (int64_t i = 0; i < n; ++i) out[i] = (int32_t)(hashes[i] % (uint64_t)nparts);
}

}  // namespace nsdb_rt
