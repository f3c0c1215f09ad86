// netsdb_amd host runtime (no torch dependency). Reference counterparts:
//   TCAP parser      <- src/logicalPlan/source/{Lexer.l,Parser.y,ParserHelperFunctions.cc}
//   BufferManager    <- src/bufferMgr (MyDB_BufferManager, LRU, pin/unpin) + src/storage/PageCache.cc
//   PartitionedFile  <- src/storage/{PartitionedFile,SequenceFile,PDBFile}.cc
//   SlabAllocator    <- src/memory/{SlabAllocator,tlsf}.cc (here: best-fit with coalescing, used for
//                       the HBM arena offsets of device-resident pages)
//   hashing          <- src/lambdas/LambdaCreationFunctions.cc mapToPartitionId, HashPartitionSink
//   WorkerQueue      <- src/work (PDBWorkerQueue, PDBWorker, PDBWork, PDBBuzzer): a fixed pool of
//                       native threads running storage work (page prefetch / flush) off the Python thread
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <deque>
#include <functional>
#include <list>
#include <memory>
#include <thread>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace nsdb_rt {

// ------------------------------------------------------------------ TCAP
struct TupleSpec {
  std::string name;
  std::vector<std::string> atts;
};

struct AtomicComputation {
  std::string type;          // APPLY FILTER HASHLEFT HASHRIGHT HASHONE FLATTEN JOIN AGGREGATE PARTITION SCAN OUTPUT
  TupleSpec output;
  TupleSpec input, projection;       // first input
  TupleSpec input2, projection2;     // JOIN right side
  std::string comp, lambda, db, set;
  int line = 0;
};

std::vector<AtomicComputation> parse_tcap(const std::string& text);  // throws std::runtime_error

// ------------------------------------------------------------------ slab allocator
class SlabAllocator {
 public:
  SlabAllocator(uint64_t capacity, uint64_t alignment);
  int64_t alloc(uint64_t bytes);   // offset or -1
  void free(int64_t offset);
  uint64_t capacity() const { return cap_; }
  uint64_t used() const { return used_; }
  uint64_t largest_free() const;
  size_t num_allocations() const { return live_.size(); }

 private:
  uint64_t cap_, align_, used_ = 0;
  std::map<uint64_t, uint64_t> free_;             // offset -> size (ordered for coalescing)
  std::multimap<uint64_t, uint64_t> by_size_;     // size -> offset
  std::unordered_map<uint64_t, uint64_t> live_;   // offset -> size
  void insert_free(uint64_t off, uint64_t sz);
  void erase_free(uint64_t off, uint64_t sz);
  mutable std::mutex mu_;
};

// ------------------------------------------------------------------ partitioned page file
class PageFile {
 public:
  PageFile(const std::string& path, uint64_t page_size);
  ~PageFile();
  void write_page(uint64_t page_no, const void* data, uint64_t bytes);
  uint64_t read_page(uint64_t page_no, void* out, uint64_t cap) const;   // returns stored bytes
  bool has_page(uint64_t page_no) const;
  std::vector<uint64_t> pages() const;
  uint64_t page_size() const { return page_size_; }
  void sync();
  const std::string& path() const { return path_; }

 private:
  std::string path_;
  uint64_t page_size_;
  int fd_ = -1;
  std::map<uint64_t, uint64_t> lengths_;   // page_no -> bytes used
  void save_meta();
  void load_meta();
  mutable std::mutex mu_;
};

// ------------------------------------------------------------------ buffer manager
struct PageKey {
  int64_t set_id;
  int64_t page_no;
  bool operator==(const PageKey& o) const { return set_id == o.set_id && page_no == o.page_no; }
};
struct PageKeyHash {
  size_t operator()(const PageKey& k) const { return std::hash<int64_t>()(k.set_id * 1000003 ^ k.page_no); }
};

class BufferManager {
 public:
  BufferManager(uint64_t page_size, uint64_t num_pages, const std::string& spill_dir);
  ~BufferManager();
  uint64_t page_size() const { return page_size_; }
  uint64_t num_slots() const { return num_slots_; }
  // pin a page: returns slot; loads from the set's file when it was evicted; allocates when new.
  int64_t pin(int64_t set_id, int64_t page_no, bool create);
  void unpin(int64_t set_id, int64_t page_no, bool dirty, uint64_t bytes_used);
  void drop_set(int64_t set_id);
  bool drop_page(int64_t set_id, int64_t page_no);   // forget one page (frame freed; file bytes left unreferenced)
  void flush_set(int64_t set_id);
  void flush_all();
  bool prefetch(int64_t set_id, int64_t page_no);   // load an evicted page into a slot (stays unpinned)
  uint8_t* slot_ptr(int64_t slot);
  uint64_t bytes_used(int64_t set_id, int64_t page_no) const;
  int64_t resident_pages() const;
  int64_t evictions() const { return evictions_; }
  int64_t loads() const { return loads_; }
  std::vector<int64_t> set_pages(int64_t set_id) const;
  std::string spill_dir() const { return dir_; }

 private:
  struct Frame {
    PageKey key{-1, -1};
    int pins = 0;
    bool dirty = false;
    uint64_t used = 0;
    std::list<int64_t>::iterator lru_it;
    bool in_lru = false;
  };
  uint64_t page_size_, num_slots_;
  std::string dir_;
  uint8_t* arena_ = nullptr;
  std::vector<Frame> frames_;
  std::vector<int64_t> free_slots_;
  std::list<int64_t> lru_;                       // unpinned resident frames, front = oldest
  std::unordered_map<PageKey, int64_t, PageKeyHash> table_;
  std::unordered_map<int64_t, PageFile*> files_;
  std::unordered_map<int64_t, std::map<int64_t, uint64_t>> known_;   // set -> page -> bytes (incl. on disk)
  int64_t evictions_ = 0, loads_ = 0;
  mutable std::mutex mu_;
  PageFile* file_for(int64_t set_id);
  int64_t grab_slot();
  void write_back(int64_t slot);
};

// ------------------------------------------------------------------ work queue
// PDBBuzzer: completion handle of one submitted work item.
class Buzzer {
 public:
  void buzz(const std::string& error = "");
  bool wait(double timeout_s);             // true when done (timeout_s < 0: wait forever)
  bool done() const;
  std::string error() const;

 private:
  mutable std::mutex mu_;
  std::condition_variable cv_;
  bool done_ = false;
  std::string error_;
};

// PDBWorkerQueue: N worker threads draining a FIFO of work items.
class WorkerQueue {
 public:
  explicit WorkerQueue(int num_workers);
  ~WorkerQueue();
  std::shared_ptr<Buzzer> submit(std::function<void()> work);
  void drain();                            // wait until every submitted item finished
  int num_workers() const { return (int)threads_.size(); }
  int64_t completed() const { return completed_.load(); }
  int64_t pending() const;

 private:
  struct Item {
    std::function<void()> fn;
    std::shared_ptr<Buzzer> buzzer;
  };
  void loop();
  std::vector<std::thread> threads_;
  std::deque<Item> q_;
  mutable std::mutex mu_;
  std::condition_variable cv_, idle_cv_;
  bool stop_ = false;
  int active_ = 0;
  std::atomic<int64_t> completed_{0};
};

// ------------------------------------------------------------------ hashing
uint64_t hash64(uint64_t x);
void hash_columns(const int64_t* const* cols, int ncols, int64_t n, uint64_t* out);
void partition_ids(const uint64_t* hashes, int64_t n, int nparts, int32_t* out);

}  // namespace nsdb_rt
