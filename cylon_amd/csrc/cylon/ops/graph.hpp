// Streaming op-graph runtime (C24).
//
// Reference: cpp/src/cylon/ops/api/parallel_op.hpp:32-183 (Op with per-tag input
// queues, children, finalize protocol), ops/execution/execution.hpp:13-95
// (RoundRobin / Priority / Sequential / Join schedulers), ops/dis_join_op.cpp,
// dis_union_op.cpp, partition_op.cpp, all_to_all_op.cpp, split_op.cpp,
// join_op.cpp, union_op.cpp, merge_op.cpp.
//
// MI355X design: every op body is a device operator from this engine (hash
// partition K1-K3, join K4-K7, union K10); the exchange edge (AllToAllOp)
// streams: each input batch becomes one exchange round (size exchange + per-buffer
// RCCL all-to-alls left in flight), polled without blocking, so batch k is split /
// joined while batch k+1 is on xGMI.  Rounds are collective and identical on every
// rank (see AllToAllOp).  The sub-partition fan-out (SplitOp) bounds the size of
// each local join like the reference's two-level partitioning.
#pragma once
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <queue>
#include <vector>

#include "../table.hpp"

namespace cylon {
namespace graph {

using ResultsCallback = std::function<void(int tag, const TablePtr &table)>;

class Op {
 public:
  Op(std::shared_ptr<CylonContext> ctx, int id, ResultsCallback callback);
  virtual ~Op() = default;

  Op *AddChild(std::shared_ptr<Op> child);
  void InsertTable(int tag, const TablePtr &table);
  // progress: run Execute on queued inputs; finalize once all parents are done and queues drained
  virtual bool IsComplete();
  bool DidSomeWork() const { return did_work_; }
  int GetId() const { return id_; }
  const std::vector<std::shared_ptr<Op>> &Children() const { return children_; }

  // external (root) completion signal
  void MarkInputsFinished();

 protected:
  virtual bool Execute(int tag, const TablePtr &table) = 0;
  virtual void OnParentsFinalized() {}
  virtual bool Finalize() { return true; }
  void InsertToAllChildren(int tag, const TablePtr &table);
  void InsertToChild(int child_id, int tag, const TablePtr &table);
  void Emit(int tag, const TablePtr &table);  // children, or the callback at a leaf

  std::shared_ptr<CylonContext> ctx_;
  int id_;

 private:
  void ReportParentCompleted();
  std::map<int, std::queue<TablePtr>> queues_;
  int64_t inputs_ = 0;
  std::vector<std::shared_ptr<Op>> children_;
  ResultsCallback callback_;
  int parents_ = 0;
  int finalized_parents_ = 0;
  bool external_root_ = true;
  bool all_parents_finalized_ = false;
  bool finalized_ = false;
  bool did_work_ = true;
};

// ---- schedulers -------------------------------------------------------------
class Execution {
 public:
  virtual ~Execution() = default;
  virtual bool IsComplete() = 0;
  // Drives the graph to completion.  Every op body is synchronous, so a graph that
  // is not complete after a bounded number of scheduler sweeps is stuck (e.g. a
  // parent that never finalizes): report it instead of spinning forever like the
  // reference's busy loop (execution.hpp:18-22).
  void WaitForCompletion(int64_t max_sweeps = int64_t(1) << 24) {
    for (int64_t i = 0; i < max_sweeps; ++i)
      if (IsComplete()) return;
    CYLON_THROW(Code::ExecutionError, "op graph made no progress after " << max_sweeps << " scheduler sweeps");
  }
};

class RoundRobinExecution : public Execution {
 public:
  void AddOp(Op *op) { ops_.push_back(op); }
  bool IsComplete() override;

 private:
  std::vector<Op *> ops_;
  size_t current_ = 0;
};

class PriorityExecution : public Execution {
 public:
  void AddOp(Op *op, int priority) { ops_.emplace_back(op, priority); }
  bool IsComplete() override;

 private:
  std::vector<std::pair<Op *, int>> ops_;
};

// breadth-first over the graph from the root, completing each op in turn
class SequentialExecution : public Execution {
 public:
  explicit SequentialExecution(Op *root);
  bool IsComplete() override;

 private:
  std::vector<Op *> order_;
  size_t current_ = 0;
};

// left subtree to completion, then the right subtree, then the join op
class JoinExecution : public Execution {
 public:
  JoinExecution(std::vector<Op *> left, std::vector<Op *> right, Op *join) : l_(left), r_(right), join_(join) {}
  bool IsComplete() override;

 private:
  std::vector<Op *> l_, r_;
  Op *join_;
  int stage_ = 0;
  size_t idx_ = 0;
};

// ---- concrete ops ----------------------------------------------------------
class RootOp : public Op {
 public:
  using Op::Op;
  void SetExecution(std::unique_ptr<Execution> e) { exec_ = std::move(e); }
  Execution *GetExecution() { return exec_.get(); }
  void WaitForCompletion() {
    MarkInputsFinished();
    exec_->WaitForCompletion();
  }

 protected:
  bool Execute(int tag, const TablePtr &table) override;

 private:
  std::unique_ptr<Execution> exec_;
};

// hash-partitions each batch into world-size partitions; emits (tag = target rank)
class PartitionOp : public Op {
 public:
  PartitionOp(std::shared_ptr<CylonContext> ctx, int id, ResultsCallback cb, std::vector<int> hash_cols);

 protected:
  bool Execute(int tag, const TablePtr &table) override;

 private:
  std::vector<int> cols_;
};

// Streaming exchange edge (reference all_to_all_op.cpp:40-62 inserts every batch into
// its ArrowAllToAll and progresses it inside IsComplete).  Here the exchange advances in
// ROUNDS that every rank takes part in, so the collectives stay matched:
//   * a round starts as soon as a whole batch has arrived (one partition per target,
//     PartitionOp emits exactly that): one all-reduce of the "inputs finished" flag,
//     then the batch's size exchange and its column all-to-alls are POSTED, not waited;
//   * IsComplete polls the posted rounds in order and emits each received table as
//     soon as its transfers have landed, while later batches are still partitioned
//     and on the wire (RCCL: its own stream; requests tested without blocking);
//   * after its own inputs end, a rank keeps joining rounds with empty sends until
//     the all-reduced flag says every rank is done.
// Only one exchange op may be progressing at a time in a schedule (JoinExecution runs
// the left subtree, then the right), which keeps the round sequence identical on all
// ranks.
class AllToAllOp : public Op {
 public:
  AllToAllOp(std::shared_ptr<CylonContext> ctx, int id, ResultsCallback cb, int out_tag);
  bool IsComplete() override;
  int64_t rounds() const { return rounds_; }
  int64_t emitted_early() const { return emitted_early_; }

 protected:
  bool Execute(int tag, const TablePtr &table) override;
  bool Finalize() override;

 private:
  bool Round(bool done);  // returns true when every rank reported done (no exchange posted)
  void Poll(bool wait);
  std::vector<std::deque<TablePtr>> per_target_;
  std::deque<std::shared_ptr<ops::PostedExchange>> posted_;
  TablePtr tmpl_;
  int out_tag_;
  bool all_done_ = false;
  int64_t rounds_ = 0, emitted_early_ = 0;
};

// local hash split into `num_splits` sub-partitions (tag = base_tag + i)
class SplitOp : public Op {
 public:
  SplitOp(std::shared_ptr<CylonContext> ctx, int id, ResultsCallback cb, int num_splits, std::vector<int> cols,
          int base_tag);

 protected:
  bool Execute(int tag, const TablePtr &table) override;

 private:
  int splits_;
  std::vector<int> cols_;
  int base_tag_;
};

// collects left / right sub-partitions and joins matching pairs at finalize
class JoinOp : public Op {
 public:
  JoinOp(std::shared_ptr<CylonContext> ctx, int id, ResultsCallback cb, join::config::JoinConfig cfg,
         int left_base_tag, int right_base_tag, int num_splits);

 protected:
  bool Execute(int tag, const TablePtr &table) override;
  bool Finalize() override;

 private:
  join::config::JoinConfig cfg_;
  int lbase_, rbase_, splits_;
  std::map<int, std::vector<TablePtr>> left_, right_;
};

class UnionOp : public Op {
 public:
  using Op::Op;

 protected:
  bool Execute(int tag, const TablePtr &table) override;
  bool Finalize() override;

 private:
  std::vector<TablePtr> tables_;
};

class MergeOp : public Op {
 public:
  using Op::Op;

 protected:
  bool Execute(int tag, const TablePtr &table) override;
  bool Finalize() override;

 private:
  std::vector<TablePtr> tables_;
};

// ---- composite roots ---------------------------------------------------------
struct DisJoinOpConfig {
  int num_splits = 16;
  join::config::JoinConfig join_config;
};

class DisJoinOP : public RootOp {
 public:
  static constexpr int kLeftTag = 100;
  static constexpr int kRightTag = 200;
  DisJoinOP(std::shared_ptr<CylonContext> ctx, int id, ResultsCallback cb, const DisJoinOpConfig &cfg);

 protected:
  bool Execute(int tag, const TablePtr &table) override;
};

class DisUnionOp : public RootOp {
 public:
  DisUnionOp(std::shared_ptr<CylonContext> ctx, int id, ResultsCallback cb);

 protected:
  bool Execute(int tag, const TablePtr &table) override;
};

}  // namespace graph
}  // namespace cylon
