// kf_stream.h — native ingest runtime: pinned host ring + reader threads +
// async H2D on a caller-provided HIP stream.
#pragma once
#include <pybind11/pybind11.h>

void bind_stream(pybind11::module_& m);
