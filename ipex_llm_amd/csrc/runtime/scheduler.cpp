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
// Exposed to Python as torch.classes.ipex_llm_amd.Scheduler.
#include <torch/custom_class.h>
#include <torch/library.h>

#include <algorithm>
#include <cstdint>
#include <deque>
#include <unordered_map>
#include <vector>

namespace {

enum State : int64_t { WAITING = 0, RUNNING = 1, FINISHED = 2, FAILED = 3 };

struct Seq {
  int64_t id = 0;
  int64_t context = 0;     // tokens that must be in the KV cache before decoding (prompt [+ generated])
  int64_t cached = 0;      // tokens whose K/V are in the cache
  int64_t admitted = 0;    // admission counter (preemption picks the latest)
  int64_t state = WAITING;
  int64_t preemptions = 0;
  std::vector<int64_t> blocks;
};

class Scheduler : public torch::CustomClassHolder {
 public:
  Scheduler(int64_t num_blocks, int64_t block_size, int64_t max_batch, int64_t max_prefill_tokens)
      : bs_(block_size), max_batch_(max_batch), max_prefill_(max_prefill_tokens) {
    TORCH_CHECK(num_blocks > 0 && block_size > 0 && max_batch > 0, "Scheduler: bad sizes");
    free_.reserve(num_blocks);
    for (int64_t b = num_blocks - 1; b >= 0; b--) free_.push_back(b);
    total_ = num_blocks;
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
        if (!free_.empty()) {
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
      if (need > (int64_t)free_.size() || (s.context > budget && !prefill.empty())) break;
      waiting_.pop_front();
      for (int64_t i = 0; i < need; i++) s.blocks.push_back(pop_free());
      s.state = RUNNING;
      s.cached = 0;
      s.admitted = ++admit_counter_;
      running_.push_back(s.id);
      prefill.push_back(s.id);
      budget -= s.context;
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
  int64_t num_free_blocks() { return (int64_t)free_.size(); }
  int64_t num_waiting() { return (int64_t)waiting_.size(); }
  int64_t num_running() { return (int64_t)running_.size(); }
  int64_t block_size() { return bs_; }

 private:
  int64_t blocks_for(int64_t tokens) const { return (tokens + bs_ - 1) / bs_; }
  bool need_block(const Seq& s) const { return s.cached + 1 > (int64_t)s.blocks.size() * bs_; }
  int64_t pop_free() {
    const int64_t b = free_.back();
    free_.pop_back();
    return b;
  }
  void release(Seq& s) {
    for (auto it = s.blocks.rbegin(); it != s.blocks.rend(); ++it) free_.push_back(*it);
    s.blocks.clear();
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
