// Tensor allocation with the GIL released (Checkpointer.materialize).
//
// A successor that materializes its state group by group allocates on a background thread
// while its main thread restores the groups already allocated.  An allocation of HBM that its
// predecessor has only just freed blocks inside the driver until the memory is cleared --
// measured on MI355X, up to 15 s behind a 170 GB spill -- and torch.empty() holds the GIL
// all that time, so the restoring thread could not even return from its (GIL-free) engine
// call.  at::empty here is the same caching-allocator allocation, without the GIL.
#include <torch/extension.h>

#include <vector>

namespace {

at::Tensor empty_nogil(const std::vector<int64_t>& shape, const at::Tensor& like) {
  const at::TensorOptions options = like.options();
  py::gil_scoped_release nogil;
  return at::empty(shape, options);
}

}  // namespace

PYBIND11_MODULE(_tpi_torch, m) {
  m.doc() = "torch helpers that release the GIL (terraform_provider_iterative_amd)";
  m.def("empty", &empty_nogil, "at::empty(shape, like.options()) with the GIL released",
        py::arg("shape"), py::arg("like"));
}
