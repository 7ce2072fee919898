// Join configuration (reference: cpp/src/cylon/join/join_config.hpp:26-189).
// Default algorithm is SORT as in the reference; on MI355X both algorithms
// are device kernels (hash: K5 open-addressing multimap, sort: K6 radix sort +
// K7 merge expansion).  Unlike the reference (its size check reads moved-from
// vectors, join_config.hpp:63-71) the key-count check here is effective.
#pragma once
#include <string>
#include <vector>

#include "../common.hpp"

namespace cylon {
namespace join {
namespace config {

enum JoinType { INNER = 0, LEFT = 1, RIGHT = 2, FULL_OUTER = 3 };
enum JoinAlgorithm { SORT = 0, HASH = 1 };

class JoinConfig {
 public:
  JoinConfig(JoinType type, int left_column_idx, int right_column_idx, JoinAlgorithm algorithm = SORT,
             std::string left_table_prefix = "", std::string right_table_prefix = "")
      : JoinConfig(type, std::vector<int>{left_column_idx}, std::vector<int>{right_column_idx}, algorithm,
                   std::move(left_table_prefix), std::move(right_table_prefix)) {}

  JoinConfig(JoinType type, std::vector<int> left_column_idx, std::vector<int> right_column_idx,
             JoinAlgorithm algorithm = SORT, std::string left_table_prefix = "",
             std::string right_table_prefix = "")
      : type_(type),
        algorithm_(algorithm),
        left_column_idx_(std::move(left_column_idx)),
        right_column_idx_(std::move(right_column_idx)),
        left_prefix_(std::move(left_table_prefix)),
        right_prefix_(std::move(right_table_prefix)) {
    CYLON_CHECK(left_column_idx_.size() == right_column_idx_.size(), Code::Invalid,
                "left and right column indices sizes are not equal");
    CYLON_CHECK(!left_column_idx_.empty(), Code::Invalid, "join needs at least one key column");
  }

#define CYLON_JOIN_FACTORY(NAME, TYPE)                                                                        \
  static JoinConfig NAME(int l, int r, JoinAlgorithm a = SORT, std::string lp = "", std::string rp = "") {   \
    return JoinConfig(TYPE, l, r, a, std::move(lp), std::move(rp));                                         \
  }                                                                                                          \
  static JoinConfig NAME(std::vector<int> l, std::vector<int> r, JoinAlgorithm a = SORT, std::string lp = "", \
                         std::string rp = "") {                                                              \
    return JoinConfig(TYPE, std::move(l), std::move(r), a, std::move(lp), std::move(rp));                   \
  }
  CYLON_JOIN_FACTORY(InnerJoin, INNER)
  CYLON_JOIN_FACTORY(LeftJoin, LEFT)
  CYLON_JOIN_FACTORY(RightJoin, RIGHT)
  CYLON_JOIN_FACTORY(FullOuterJoin, FULL_OUTER)
#undef CYLON_JOIN_FACTORY

  JoinType GetType() const { return type_; }
  JoinAlgorithm GetAlgorithm() const { return algorithm_; }
  const std::vector<int> &GetLeftColumnIdx() const { return left_column_idx_; }
  const std::vector<int> &GetRightColumnIdx() const { return right_column_idx_; }
  const std::string &GetLeftTableSuffix() const { return left_prefix_; }
  const std::string &GetRightTableSuffix() const { return right_prefix_; }
  const std::string &GetLeftTablePrefix() const { return left_prefix_; }
  const std::string &GetRightTablePrefix() const { return right_prefix_; }
  bool IsMultiColumn() const { return left_column_idx_.size() > 1; }

 private:
  JoinType type_;
  JoinAlgorithm algorithm_;
  std::vector<int> left_column_idx_;
  std::vector<int> right_column_idx_;
  std::string left_prefix_;
  std::string right_prefix_;
};

}  // namespace config
}  // namespace join
}  // namespace cylon
