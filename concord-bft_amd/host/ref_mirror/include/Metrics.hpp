// Standalone-build restatement of the part of the reference's metrics library that SigManager
// uses (util/include/Metrics.hpp:36-38,56-83,108-131,214-318; util/src/Metrics.cpp): a Component
// owns counters and pushes a snapshot of them to its Aggregator on UpdateAggregator(); callers
// read the Aggregator (the reference's MetricsServer / Apollo tests read counters the same way).
// Handles index into the component's value vector, as there.  See ../README.md.
#pragma once

#include <atomic>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace concordMetrics {

template <class T>
class BasicCounter {
 public:
  using type = uint64_t;
  BasicCounter() : val_(0) {}
  explicit BasicCounter(const uint64_t val) : val_(val) {}
  BasicCounter(const BasicCounter& c) { val_ = (uint64_t)c.val_; }
  BasicCounter& operator=(const BasicCounter& c) {
    val_ = (uint64_t)c.val_;
    return *this;
  }
  BasicCounter operator++(int) { return BasicCounter(val_++); }
  BasicCounter& operator+=(const uint64_t& rhs) {
    val_ += rhs;
    return *this;
  }
  T& Get() { return val_; }

 private:
  T val_;
};

using Counter = BasicCounter<uint64_t>;
using AtomicCounter = BasicCounter<std::atomic_uint64_t>;

class Component;

class Aggregator {
 public:
  explicit Aggregator(bool metricsEnabled = true) : metricsEnabled_(metricsEnabled) {}
  // The last pushed value of component_name.val_name (throws std::invalid_argument if unknown).
  Counter GetCounter(const std::string& component_name, const std::string& val_name);
  // Number of UpdateAggregator() pushes received from component_name (restatement diagnostics).
  uint64_t Pushes(const std::string& component_name);

 private:
  friend class Component;
  void RegisterComponent(Component& component);
  void UpdateValues(const std::string& name, const std::vector<std::pair<std::string, uint64_t>>& values);

  std::mutex lock_;
  std::map<std::string, std::map<std::string, uint64_t>> counters_;
  std::map<std::string, uint64_t> pushes_;
  const bool metricsEnabled_;
};

class Component {
 public:
  template <typename T>
  class Handle {
   public:
    Handle(std::vector<T>& values, size_t index, bool metricsEnabled)
        : values_(values), index_(index), metricsEnabled_(metricsEnabled) {}
    T& Get() { return values_[index_]; }
    T operator++(int) {
      if (!metricsEnabled_) return Get();
      return Get()++;
    }
    T& operator+=(const typename T::type& rhs) {
      if (!metricsEnabled_) return Get();
      Get() += rhs;
      return Get();
    }

   private:
    std::vector<T>& values_;
    size_t index_;
    const bool metricsEnabled_;
  };

  Component(const std::string& name, std::shared_ptr<Aggregator> aggregator)
      : aggregator_(aggregator), name_(name), metricsEnabled_(aggregator->metricsEnabled_) {
    atomic_counters_.reserve(64);  // handles index into the vector: no reallocation after registration
  }
  std::string Name() { return name_; }
  Handle<AtomicCounter> RegisterAtomicCounter(const std::string& name, const uint64_t val);
  Handle<AtomicCounter> RegisterAtomicCounter(const std::string& name) { return RegisterAtomicCounter(name, 0); }
  void Register() {
    if (auto a = aggregator_.lock()) a->RegisterComponent(*this);
  }
  // Pushes the current values to the aggregator.
  void UpdateAggregator();
  void SetAggregator(std::shared_ptr<Aggregator> aggregator) {
    aggregator_ = aggregator;
    Register();
  }

 private:
  friend class Aggregator;
  std::weak_ptr<Aggregator> aggregator_;
  const std::string name_;
  const bool metricsEnabled_;
  std::vector<std::string> atomic_counter_names_;
  std::vector<AtomicCounter> atomic_counters_;
};

typedef Component::Handle<AtomicCounter> AtomicCounterHandle;

}  // namespace concordMetrics
