// Registration hook for the operator bindings that live outside bindings.cpp
// (set operations, group-by, aggregates, indexing, ...).
#pragma once
#include <pybind11/pybind11.h>

void register_extended_ops(pybind11::module &m);
