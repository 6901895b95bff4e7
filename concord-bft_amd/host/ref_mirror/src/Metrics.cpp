// Standalone-build restatement of util/src/Metrics.cpp (the counter path; see Metrics.hpp).
#include "Metrics.hpp"

#include <stdexcept>

namespace concordMetrics {

Counter Aggregator::GetCounter(const std::string& component_name, const std::string& val_name) {
  std::lock_guard<std::mutex> g(lock_);
  auto c = counters_.find(component_name);
  if (c == counters_.end()) throw std::invalid_argument("Invalid component name: " + component_name);
  auto v = c->second.find(val_name);
  if (v == c->second.end()) throw std::invalid_argument("Invalid counter name: " + val_name);
  return Counter(v->second);
}

uint64_t Aggregator::Pushes(const std::string& component_name) {
  std::lock_guard<std::mutex> g(lock_);
  auto it = pushes_.find(component_name);
  return it == pushes_.end() ? 0 : it->second;
}

void Aggregator::RegisterComponent(Component& component) {
  std::vector<std::pair<std::string, uint64_t>> vals;
  for (size_t i = 0; i < component.atomic_counters_.size(); i++)
    vals.emplace_back(component.atomic_counter_names_[i], (uint64_t)component.atomic_counters_[i].Get());
  std::lock_guard<std::mutex> g(lock_);
  auto& m = counters_[component.name_];
  for (auto& [n, v] : vals) m[n] = v;
}

void Aggregator::UpdateValues(const std::string& name, const std::vector<std::pair<std::string, uint64_t>>& values) {
  std::lock_guard<std::mutex> g(lock_);
  auto& m = counters_[name];
  for (auto& [n, v] : values) m[n] = v;
  pushes_[name]++;
}

Component::Handle<AtomicCounter> Component::RegisterAtomicCounter(const std::string& name, const uint64_t val) {
  if (atomic_counters_.size() == atomic_counters_.capacity())
    throw std::length_error("Component: too many counters");  // handles must stay valid
  atomic_counter_names_.push_back(name);
  atomic_counters_.emplace_back(val);
  return Handle<AtomicCounter>(atomic_counters_, atomic_counters_.size() - 1, metricsEnabled_);
}

void Component::UpdateAggregator() {
  auto a = aggregator_.lock();
  if (!a) return;
  std::vector<std::pair<std::string, uint64_t>> vals;
  vals.reserve(atomic_counters_.size());
  for (size_t i = 0; i < atomic_counters_.size(); i++)
    vals.emplace_back(atomic_counter_names_[i], (uint64_t)atomic_counters_[i].Get());
  a->UpdateValues(name_, vals);
}

}  // namespace concordMetrics
