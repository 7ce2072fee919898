// Op-graph runtime implementation (see graph.hpp).
#include "graph.hpp"

#include "relational.hpp"
#include "util.hpp"
#include "../trace.hpp"

namespace cylon {
namespace graph {

// ---------------------------------------------------------------------------
// Op
// ---------------------------------------------------------------------------
Op::Op(std::shared_ptr<CylonContext> ctx, int id, ResultsCallback callback)
    : ctx_(std::move(ctx)), id_(id), callback_(std::move(callback)) {}

Op *Op::AddChild(std::shared_ptr<Op> child) {
  child->parents_++;
  child->external_root_ = false;
  children_.push_back(child);
  return this;
}

void Op::InsertTable(int tag, const TablePtr &table) {
  queues_[tag].push(table);
  inputs_++;
}

void Op::MarkInputsFinished() { finalized_parents_ = parents_ + 1; }

void Op::ReportParentCompleted() { finalized_parents_++; }

void Op::InsertToAllChildren(int tag, const TablePtr &table) {
  for (auto &c : children_) c->InsertTable(tag, table);
}

void Op::InsertToChild(int child_id, int tag, const TablePtr &table) {
  for (auto &c : children_)
    if (c->GetId() == child_id) {
      c->InsertTable(tag, table);
      return;
    }
  CYLON_THROW(Code::KeyError, "op " << id_ << " has no child " << child_id);
}

void Op::Emit(int tag, const TablePtr &table) {
  if (children_.empty()) {
    if (callback_) callback_(tag, table);
  } else {
    InsertToAllChildren(tag, table);
  }
}

bool Op::IsComplete() {
  did_work_ = false;
  for (auto &kv : queues_) {
    auto &q = kv.second;
    while (!q.empty()) {
      if (!Execute(kv.first, q.front())) break;
      q.pop();
      inputs_--;
      did_work_ = true;
    }
  }
  if (!finalized_) {
    // a root (no graph parents) finishes after MarkInputsFinished(); others after all parents finalized
    const bool parents_done = external_root_ ? finalized_parents_ > parents_ : finalized_parents_ >= parents_;
    if (parents_done && inputs_ == 0) {
      if (!all_parents_finalized_) {
        all_parents_finalized_ = true;
        OnParentsFinalized();
        did_work_ = true;
      }
      if (inputs_ == 0 && Finalize()) {
        finalized_ = true;
        for (auto &c : children_) c->ReportParentCompleted();
        did_work_ = true;
      }
    }
  }
  return finalized_;
}

// ---------------------------------------------------------------------------
// schedulers
// ---------------------------------------------------------------------------
bool RoundRobinExecution::IsComplete() {
  bool all = true;
  for (auto *op : ops_) all &= op->IsComplete();
  return all;
}

bool PriorityExecution::IsComplete() {
  bool all = true;
  for (auto &p : ops_) {
    bool done = false;
    for (int i = 0; i < std::max(1, p.second); ++i) {
      done = p.first->IsComplete();
      if (done || !p.first->DidSomeWork()) break;
    }
    all &= done;
  }
  return all;
}

SequentialExecution::SequentialExecution(Op *root) {
  std::vector<Op *> frontier{root};
  while (!frontier.empty()) {
    std::vector<Op *> next;
    for (Op *op : frontier) {
      bool seen = false;
      for (Op *o : order_) seen |= (o == op);
      if (seen) continue;
      order_.push_back(op);
      for (auto &c : op->Children()) next.push_back(c.get());
    }
    frontier = std::move(next);
  }
}

bool SequentialExecution::IsComplete() {
  while (current_ < order_.size()) {
    // ops before `current_` are finalized; keep them ticking so their children get inputs
    if (!order_[current_]->IsComplete()) return false;
    ++current_;
  }
  return true;
}

bool JoinExecution::IsComplete() {
  // the ops of one subtree are progressed round-robin (a batch flows root -> partition ->
  // exchange -> split while the next one follows), one subtree at a time
  auto run = [](std::vector<Op *> &ops, size_t &) {
    bool all = true;
    for (Op *op : ops) all &= op->IsComplete();
    return all;
  };
  if (stage_ == 0) {
    if (!run(l_, idx_)) return false;
    stage_ = 1;
    idx_ = 0;
  }
  if (stage_ == 1) {
    if (!run(r_, idx_)) return false;
    stage_ = 2;
  }
  return join_->IsComplete();
}

// ---------------------------------------------------------------------------
// ops
// ---------------------------------------------------------------------------
bool RootOp::Execute(int tag, const TablePtr &table) {
  InsertToAllChildren(tag, table);
  return true;
}

PartitionOp::PartitionOp(std::shared_ptr<CylonContext> ctx, int id, ResultsCallback cb, std::vector<int> hash_cols)
    : Op(std::move(ctx), id, std::move(cb)), cols_(std::move(hash_cols)) {}

bool PartitionOp::Execute(int, const TablePtr &table) {
  const int world = ctx_->GetWorldSize();
  if (!ctx_->ShuffleRequired()) {
    Emit(0, table);
    return true;
  }
  std::vector<int> cols = cols_;
  if (cols.empty())  // all columns (set operations)
    for (int i = 0; i < table->Columns(); ++i) cols.push_back(i);
  auto parts = ops::HashPartition(table, cols, (uint32_t)world);
  for (int i = 0; i < world; ++i) Emit(i, parts[i]);
  return true;
}

AllToAllOp::AllToAllOp(std::shared_ptr<CylonContext> ctx, int id, ResultsCallback cb, int out_tag)
    : Op(std::move(ctx), id, std::move(cb)), out_tag_(out_tag) {
  per_target_.resize(ctx_->GetWorldSize());
}

bool AllToAllOp::Execute(int tag, const TablePtr &table) {
  CYLON_CHECK(tag >= 0 && tag < (int)per_target_.size(), Code::IndexError, "all-to-all target " << tag);
  per_target_[tag].push_back(table);
  if (!tmpl_) tmpl_ = table;
  bool whole = true;
  for (auto &v : per_target_) whole &= !v.empty();
  if (whole) Round(false);
  Poll(false);
  return true;
}

bool AllToAllOp::Round(bool done) {
  at::Tensor flag = at::full({1}, done ? 1 : 0, at::TensorOptions().dtype(at::kInt).device(ctx_->GetDevice()));
  if (ctx_->GetWorldSize() > 1) ctx_->GetCommunicator()->AllReduce(flag, net::ReduceOp::SUM);
  if (flag.item<int>() == ctx_->GetWorldSize()) return true;
  CYLON_CHECK(tmpl_ != nullptr, Code::Invalid, "AllToAllOp on rank " << ctx_->GetRank() << " received no table");
  std::vector<TablePtr> ordered;
  std::vector<int64_t> counts;
  for (auto &v : per_target_) {  // one batch = the oldest pending partition of every target
    TablePtr m = v.empty() ? ops::Slice(tmpl_, 0, 0) : v.front();
    if (!v.empty()) v.pop_front();
    counts.push_back(m->Rows());
    ordered.push_back(m);
  }
  posted_.push_back(ops::PostAllToAllTable(ops::Merge(ordered), counts));
  ++rounds_;
  trace::add_counter("graph.alltoall.rounds", 1);
  return false;
}

void AllToAllOp::Poll(bool wait) {
  while (!posted_.empty() && (wait || ops::PostedExchangeReady(*posted_.front()))) {
    if (!wait) {
      ++emitted_early_;
      trace::add_counter("graph.alltoall.streamed_rounds", 1);  // emitted before the inputs ended
    }
    TablePtr out = ops::FinishPostedExchange(*posted_.front());
    posted_.pop_front();
    Emit(out_tag_, out);
  }
}

bool AllToAllOp::IsComplete() {
  Poll(false);
  return Op::IsComplete();
}

bool AllToAllOp::Finalize() {
  if (!all_done_) {
    for (;;) {  // batches still pending (incomplete ones included)
      bool pending = false;
      for (auto &v : per_target_) pending |= !v.empty();
      if (!pending) break;
      Round(false);
    }
    while (!Round(true)) {                     // empty rounds until every rank is done
    }
    all_done_ = true;
  }
  Poll(true);
  return true;
}

SplitOp::SplitOp(std::shared_ptr<CylonContext> ctx, int id, ResultsCallback cb, int num_splits, std::vector<int> cols,
                 int base_tag)
    : Op(std::move(ctx), id, std::move(cb)), splits_(num_splits), cols_(std::move(cols)), base_tag_(base_tag) {}

bool SplitOp::Execute(int, const TablePtr &table) {
  // independent of the rank partition: 64-bit row hash, high bits
  ops::Exec ex(table->device());
  const int64_t n = table->Rows();
  std::vector<ColView> v = ops::views(table, cols_);
  at::Tensor h = ex.empty_i64(n);
  KCALL(ex, row_hash64, v.data(), (int)v.size(), n, reinterpret_cast<uint64_t *>(ops::ptr<int64_t>(h)));
  at::Tensor pid = at::remainder(at::bitwise_right_shift(h, 33), splits_).to(at::kInt).contiguous();
  auto parts = ops::Split(table, pid, (uint32_t)splits_);
  for (int i = 0; i < splits_; ++i) Emit(base_tag_ + i, parts[i]);
  return true;
}

JoinOp::JoinOp(std::shared_ptr<CylonContext> ctx, int id, ResultsCallback cb, join::config::JoinConfig cfg,
               int left_base_tag, int right_base_tag, int num_splits)
    : Op(std::move(ctx), id, std::move(cb)),
      cfg_(std::move(cfg)),
      lbase_(left_base_tag),
      rbase_(right_base_tag),
      splits_(num_splits) {}

bool JoinOp::Execute(int tag, const TablePtr &table) {
  if (tag >= lbase_ && tag < lbase_ + splits_) left_[tag - lbase_].push_back(table);
  else if (tag >= rbase_ && tag < rbase_ + splits_) right_[tag - rbase_].push_back(table);
  else CYLON_THROW(Code::Invalid, "join op: unexpected tag " << tag);
  return true;
}

bool JoinOp::Finalize() {
  TablePtr ltmpl, rtmpl;
  for (auto &kv : left_) ltmpl = kv.second[0];
  for (auto &kv : right_) rtmpl = kv.second[0];
  if (!ltmpl || !rtmpl) return true;  // nothing to join on this rank
  std::vector<TablePtr> results;
  for (int i = 0; i < splits_; ++i) {
    TablePtr l = left_.count(i) ? ops::Merge(left_[i]) : ops::Slice(ltmpl, 0, 0);
    TablePtr r = right_.count(i) ? ops::Merge(right_[i]) : ops::Slice(rtmpl, 0, 0);
    TablePtr j = ops::Join(l, r, cfg_);
    if (j->Rows() > 0 || results.empty()) results.push_back(j);
  }
  left_.clear();
  right_.clear();
  Emit(0, ops::Merge(results));
  return true;
}

bool UnionOp::Execute(int, const TablePtr &table) {
  tables_.push_back(table);
  return true;
}

bool UnionOp::Finalize() {
  if (tables_.empty()) return true;
  TablePtr m = ops::Merge(tables_);
  tables_.clear();
  Emit(0, ops::Unique(m, {}, true));
  return true;
}

bool MergeOp::Execute(int, const TablePtr &table) {
  tables_.push_back(table);
  return true;
}

bool MergeOp::Finalize() {
  if (tables_.empty()) return true;
  Emit(0, ops::Merge(tables_));
  tables_.clear();
  return true;
}

// ---------------------------------------------------------------------------
// composites
// ---------------------------------------------------------------------------
DisJoinOP::DisJoinOP(std::shared_ptr<CylonContext> ctx, int id, ResultsCallback cb, const DisJoinOpConfig &cfg)
    : RootOp(ctx, id, nullptr) {
  const auto &jc = cfg.join_config;
  auto pl = std::make_shared<PartitionOp>(ctx, 1, nullptr, jc.GetLeftColumnIdx());
  auto pr = std::make_shared<PartitionOp>(ctx, 2, nullptr, jc.GetRightColumnIdx());
  auto al = std::make_shared<AllToAllOp>(ctx, 3, nullptr, kLeftTag);
  auto ar = std::make_shared<AllToAllOp>(ctx, 4, nullptr, kRightTag);
  auto sl = std::make_shared<SplitOp>(ctx, 5, nullptr, cfg.num_splits, jc.GetLeftColumnIdx(), kLeftTag);
  auto sr = std::make_shared<SplitOp>(ctx, 6, nullptr, cfg.num_splits, jc.GetRightColumnIdx(), kRightTag);
  auto j = std::make_shared<JoinOp>(ctx, 7, cb, jc, kLeftTag, kRightTag, cfg.num_splits);
  AddChild(pl);
  AddChild(pr);
  pl->AddChild(al);
  pr->AddChild(ar);
  al->AddChild(sl);
  ar->AddChild(sr);
  sl->AddChild(j);
  sr->AddChild(j);
  SetExecution(std::make_unique<JoinExecution>(std::vector<Op *>{this, pl.get(), al.get(), sl.get()},
                                               std::vector<Op *>{pr.get(), ar.get(), sr.get()}, j.get()));
}

bool DisJoinOP::Execute(int tag, const TablePtr &table) {
  if (tag == kLeftTag) InsertToChild(1, tag, table);
  else if (tag == kRightTag) InsertToChild(2, tag, table);
  else CYLON_THROW(Code::Invalid, "DisJoinOP accepts tags " << kLeftTag << " (left) and " << kRightTag << " (right)");
  return true;
}

DisUnionOp::DisUnionOp(std::shared_ptr<CylonContext> ctx, int id, ResultsCallback cb) : RootOp(ctx, id, nullptr) {
  auto p = std::make_shared<PartitionOp>(ctx, 1, nullptr, std::vector<int>{});
  auto a = std::make_shared<AllToAllOp>(ctx, 2, nullptr, 0);
  auto u = std::make_shared<UnionOp>(ctx, 3, cb);
  AddChild(p);
  p->AddChild(a);
  a->AddChild(u);
  auto seq = std::make_unique<SequentialExecution>(this);
  SetExecution(std::move(seq));
}

bool DisUnionOp::Execute(int tag, const TablePtr &table) {
  InsertToAllChildren(tag, table);  // partition op hashes all columns (empty hash-column list)
  return true;
}

}  // namespace graph
}  // namespace cylon
