// Continuous-batching scheduler + paged KV block manager (native runtime).
//
// Reference capability: the serving paths batch requests through vLLM's
// Python scheduler (``SRC/vllm/xpu/engine/engine.py``) or serve one request
// at a time (``SRC/serving/fastapi/model_worker.py``); the NPU runtime keeps
// its decode loop in C++ (``npu_llm_cpp.py``).  Here the
// per-step bookkeeping of a serving engine -- which sequences decode, which
// waiting requests are admitted for prefill, block allocation for every new
// token, preemption (recompute) when the KV pool is exhausted -- is C++,
// so the Python side only launches the GPU work.
//
// Policy (per ``schedule()`` call):
//   1. every RUNNING sequence gets room for its next token; when the pool is
//      empty the most recently admitted running sequence is preempted (its
//      blocks are freed, it goes back to the front of the queue and will be
//      re-prefilled with prompt + generated tokens);
//   2. WAITING requests are admitted FCFS while the batch has room, the
//      step's prefill token budget is not exceeded and the pool can hold
//      prompt + 1 tokens (a request that can never fit is failed).
//
// Automatic prefix caching (``enable_prefix_caching()``, the vLLM APC feature
// of the reference's serving stack, BASELINE "Automatic prefix caching
// demo"): every FULL block whose K/V are computed is registered under a
// chained 64-bit content hash (parent hash + its bs token ids, verified
// against the stored ids on lookup).  Blocks are reference-counted; a block
// whose last user finishes stays cached on an LRU list and is reclaimed only
// when the pool runs dry.  An admitted request (or a preempted one coming
// back) reuses the longest chain of cached blocks of its context (at least
// its last token is always recomputed, it yields the next-token logits), so
// only the uncached suffix is prefilled.  Cached blocks are immutable: new
// tokens always go to blocks past the shared full ones.
// Exposed to Python as torch.classes.ipex_llm_amd.Scheduler.
#include <torch/custom_class.h>
#include <torch/library.h>

#include <algorithm>
#include <cstdint>
#include <deque>
#include <set>
#include <unordered_map>
#include <utility>
#include <vector>

namespace {

enum State : int64_t { WAITING = 0, RUNNING = 1, FINISHED = 2, FAILED = 3 };

constexpr uint64_t kSeed = 0x9e3779b97f4a7c15ull;   // chain hash of the empty prefix

struct Seq {
  int64_t id = 0;
  int64_t context = 0;     // tokens that must be in the KV cache before decoding (prompt [+ generated])
  int64_t cached = 0;      // tokens whose K/V are in the cache
  int64_t admitted = 0;    // admission counter (preemption picks the latest)
  int64_t state = WAITING;
  int64_t preemptions = 0;
  std::vector<int64_t> blocks;
  std::vector<int64_t> toks;  // prompt + generated ids (prefix caching only)
  int64_t nhashed = 0;        // leading full blocks already hashed / registered
  uint64_t last_hash = kSeed; // chain hash after nhashed blocks
};

uint64_t hash_block(uint64_t parent, const int64_t* t, int64_t n) {
  uint64_t h = parent ^ 0xcbf29ce484222325ull;
  for (int64_t i = 0; i < n; i++) {
    uint64_t v = (uint64_t)t[i] + 0x9e3779b97f4a7c15ull;
    v = (v ^ (v >> 30)) * 0xbf58476d1ce4e5b9ull;
    v = (v ^ (v >> 27)) * 0x94d049bb133111ebull;
    h = (h ^ (v ^ (v >> 31))) * 0x100000001b3ull;
  }
  return h ? h : 1;  // 0 marks "no hash"
}

struct CachedBlock {
  int64_t block;
  uint64_t parent;
  std::vector<int64_t> toks;
};

class Scheduler : public torch::CustomClassHolder {
 public:
  Scheduler(int64_t num_blocks, int64_t block_size, int64_t max_batch, int64_t max_prefill_tokens)
      : bs_(block_size), max_batch_(max_batch), max_prefill_(max_prefill_tokens) {
    TORCH_CHECK(num_blocks > 0 && block_size > 0 && max_batch > 0, "Scheduler: bad sizes");
    free_.reserve(num_blocks);
    for (int64_t b = num_blocks - 1; b >= 0; b--) free_.push_back(b);
    total_ = num_blocks;
    ref_.assign(num_blocks, 0);
    bhash_.assign(num_blocks, 0);
    etick_.assign(num_blocks, -1);
  }

  void enable_prefix_caching(bool on) { apc_ = on; }

  // request with its prompt token ids (prefix caching needs the content)
  void add_tokens(int64_t id, std::vector<int64_t> prompt) {
    add(id, (int64_t)prompt.size());
    if (apc_) seqs_[id].toks = std::move(prompt);
  }

  // a generated token (fed next step): the context grows by one
  void append(int64_t id, int64_t tok) {
    Seq& s = get(id);
    s.context += 1;
    if (apc_) s.toks.push_back(tok);
  }

  void add(int64_t id, int64_t prompt_len) {
    TORCH_CHECK(!seqs_.count(id), "Scheduler: duplicate request id ", id);
    TORCH_CHECK(prompt_len > 0, "Scheduler: empty prompt");
    Seq s;
    s.id = id;
    s.context = prompt_len;
    seqs_[id] = s;
    waiting_.push_back(id);
  }

  // -> [prefill ids..., -1, decode ids..., -1, preempted ids..., -1, failed ids...]
  std::vector<int64_t> schedule() {
    std::vector<int64_t> prefill, decode, preempted, failed;
    // 1. room for the next token of every running sequence
    std::vector<int64_t> run(running_.begin(), running_.end());
    for (size_t i = 0; i < run.size(); i++) {
      Seq& s = seqs_[run[i]];
      if (s.state != RUNNING) continue;
      while (need_block(s)) {
        // the free list first, then idle cached (prefix) blocks: a running
        // sequence is preempted only when neither is left
        if (available() > 0) {
          s.blocks.push_back(pop_free());
          continue;
        }
        // preempt the latest-admitted running sequence (possibly s itself)
        int64_t victim = -1, best = -1;
        for (int64_t r : running_) {
          const Seq& c = seqs_[r];
          if (c.state == RUNNING && c.admitted > best) { best = c.admitted; victim = r; }
        }
        preempt(victim);
        preempted.push_back(victim);
        if (victim == s.id) break;
      }
    }
    for (int64_t r : running_)
      if (seqs_[r].state == RUNNING) decode.push_back(r);
    // 2. admit waiting requests
    int64_t budget = max_prefill_;
    while (!waiting_.empty() && (int64_t)(decode.size() + prefill.size()) < max_batch_) {
      Seq& s = seqs_[waiting_.front()];
      const int64_t need = blocks_for(s.context + 1);
      if (need > total_) {  // can never fit
        s.state = FAILED;
        failed.push_back(s.id);
        waiting_.pop_front();
        continue;
      }
      std::vector<int64_t> hit;
      uint64_t chain = kSeed;
      match_prefix(s, hit, chain);
      int64_t hit_idle = 0;  // cached blocks nobody holds: reusing them does not consume the pool
      for (int64_t b : hit) hit_idle += ref_[b] == 0;
      const int64_t fresh = need - (int64_t)hit.size();
      const int64_t todo = s.context - (int64_t)hit.size() * bs_;
      if (fresh > available() - hit_idle || (todo > budget && !prefill.empty())) break;
      waiting_.pop_front();
      for (int64_t b : hit) take(b);
      s.blocks = hit;
      for (int64_t i = 0; i < fresh; i++) s.blocks.push_back(pop_free());
      s.state = RUNNING;
      s.cached = (int64_t)hit.size() * bs_;
      s.nhashed = (int64_t)hit.size();
      s.last_hash = chain;
      hit_tokens_ += s.cached;
      s.admitted = ++admit_counter_;
      running_.push_back(s.id);
      prefill.push_back(s.id);
      budget -= todo;
    }
    std::vector<int64_t> out;
    for (auto* v : {&prefill, &decode, &preempted}) {
      out.insert(out.end(), v->begin(), v->end());
      out.push_back(-1);
    }
    out.insert(out.end(), failed.begin(), failed.end());
    return out;
  }

  // n new tokens of sequence id now have K/V in the cache
  void advance(int64_t id, int64_t n) {
    Seq& s = get(id);
    s.cached += n;
    if (s.cached > s.context) s.context = s.cached;
    TORCH_CHECK(s.cached <= (int64_t)s.blocks.size() * bs_, "Scheduler: sequence ", id, " overran its blocks");
    if (apc_) register_full_blocks(s);
  }

  // a token was generated (it will be fed next step): the context grows by one
  void grow(int64_t id) { get(id).context += 1; }

  void finish(int64_t id) {
    Seq& s = get(id);
    release(s);
    s.state = FINISHED;
    running_.erase(std::remove(running_.begin(), running_.end(), id), running_.end());
    waiting_.erase(std::remove(waiting_.begin(), waiting_.end(), id), waiting_.end());
    seqs_.erase(id);
  }

  std::vector<int64_t> blocks(int64_t id) { return get(id).blocks; }
  int64_t cached(int64_t id) { return get(id).cached; }
  int64_t context(int64_t id) { return get(id).context; }
  int64_t state(int64_t id) { return get(id).state; }
  int64_t num_free_blocks() { return available(); }
  int64_t num_cached_blocks() { return (int64_t)cache_.size(); }
  int64_t prefix_hit_tokens() { return hit_tokens_; }
  int64_t num_waiting() { return (int64_t)waiting_.size(); }
  int64_t num_running() { return (int64_t)running_.size(); }
  int64_t block_size() { return bs_; }

 private:
  int64_t blocks_for(int64_t tokens) const { return (tokens + bs_ - 1) / bs_; }
  bool need_block(const Seq& s) const { return s.cached + 1 > (int64_t)s.blocks.size() * bs_; }
  int64_t available() const { return (int64_t)(free_.size() + evict_.size()); }
  // a fresh block: the free list first, else the least recently released cached block
  int64_t pop_free() {
    int64_t b;
    if (!free_.empty()) {
      b = free_.back();
      free_.pop_back();
    } else {
      TORCH_CHECK(!evict_.empty(), "Scheduler: KV pool exhausted");
      b = evict_.begin()->second;
      evict_.erase(evict_.begin());
      etick_[b] = -1;
      cache_.erase(bhash_[b]);
      bhash_[b] = 0;
    }
    ref_[b] = 1;
    return b;
  }
  // one more holder of a cached block
  void take(int64_t b) {
    if (ref_[b] == 0 && etick_[b] >= 0) {
      evict_.erase({etick_[b], b});
      etick_[b] = -1;
    }
    ref_[b]++;
  }
  void release(Seq& s) {
    for (auto it = s.blocks.rbegin(); it != s.blocks.rend(); ++it) {
      const int64_t b = *it;
      if (--ref_[b] > 0) continue;
      if (bhash_[b] != 0) {          // keep its content for later hits (LRU)
        etick_[b] = ++tick_;
        evict_.insert({etick_[b], b});
      } else {
        free_.push_back(b);
      }
    }
    s.blocks.clear();
    s.nhashed = 0;
    s.last_hash = kSeed;
  }
  // longest chain of cached full blocks covering the context minus its last token
  void match_prefix(const Seq& s, std::vector<int64_t>& hit, uint64_t& chain) {
    chain = kSeed;
    if (!apc_ || (int64_t)s.toks.size() < s.context) return;
    const int64_t maxb = (s.context - 1) / bs_;
    for (int64_t i = 0; i < maxb; i++) {
      const int64_t* t = s.toks.data() + i * bs_;
      const uint64_t h = hash_block(chain, t, bs_);
      auto it = cache_.find(h);
      if (it == cache_.end() || it->second.parent != chain || !std::equal(t, t + bs_, it->second.toks.begin()))
        break;
      hit.push_back(it->second.block);
      chain = h;
    }
  }
  // full blocks whose K/V are now computed join the content index
  void register_full_blocks(Seq& s) {
    while ((s.nhashed + 1) * bs_ <= s.cached && (s.nhashed + 1) * bs_ <= (int64_t)s.toks.size()) {
      const int64_t i = s.nhashed;
      const int64_t* t = s.toks.data() + i * bs_;
      const uint64_t h = hash_block(s.last_hash, t, bs_);
      const int64_t b = s.blocks[i];
      if (!cache_.count(h) && bhash_[b] == 0) {
        cache_[h] = CachedBlock{b, s.last_hash, std::vector<int64_t>(t, t + bs_)};
        bhash_[b] = h;
      }
      s.last_hash = h;
      s.nhashed++;
    }
  }
  void preempt(int64_t id) {
    Seq& s = get(id);
    release(s);
    s.cached = 0;
    s.state = WAITING;
    s.preemptions++;
    running_.erase(std::remove(running_.begin(), running_.end(), id), running_.end());
    waiting_.push_front(id);
  }
  Seq& get(int64_t id) {
    auto it = seqs_.find(id);
    TORCH_CHECK(it != seqs_.end(), "Scheduler: unknown request id ", id);
    return it->second;
  }

  int64_t bs_, max_batch_, max_prefill_, total_ = 0, admit_counter_ = 0;
  std::vector<int64_t> free_;
  // prefix caching
  bool apc_ = false;
  std::unordered_map<uint64_t, CachedBlock> cache_;  // content hash -> block
  std::vector<int32_t> ref_;                          // holders per block
  std::vector<uint64_t> bhash_;                       // hash a block is registered under (0: none)
  std::vector<int64_t> etick_;                        // LRU tick of an idle cached block (-1: not idle)
  std::set<std::pair<int64_t, int64_t>> evict_;       // idle cached blocks, oldest first
  int64_t tick_ = 0, hit_tokens_ = 0;
  std::deque<int64_t> waiting_;
  std::vector<int64_t> running_;
  std::unordered_map<int64_t, Seq> seqs_;
};

}  // namespace

TORCH_LIBRARY_FRAGMENT(ipex_llm_amd, m) {
  m.class_<Scheduler>("Scheduler")
      .def(torch::init<int64_t, int64_t, int64_t, int64_t>())
      .def("add", &Scheduler::add)
      .def("schedule", &Scheduler::schedule)
      .def("advance", &Scheduler::advance)
      .def("grow", &Scheduler::grow)
      .def("enable_prefix_caching", &Scheduler::enable_prefix_caching)
      .def("add_tokens", &Scheduler::add_tokens)
      .def("append", &Scheduler::append)
      .def("num_cached_blocks", &Scheduler::num_cached_blocks)
      .def("prefix_hit_tokens", &Scheduler::prefix_hit_tokens)
      .def("finish", &Scheduler::finish)
      .def("blocks", &Scheduler::blocks)
      .def("cached", &Scheduler::cached)
      .def("context", &Scheduler::context)
      .def("state", &Scheduler::state)
      .def("num_free_blocks", &Scheduler::num_free_blocks)
      .def("num_waiting", &Scheduler::num_waiting)
      .def("num_running", &Scheduler::num_running)
      .def("block_size", &Scheduler::block_size);
}
