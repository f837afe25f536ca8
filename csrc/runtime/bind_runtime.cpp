// Python bindings of the native host runtime (kept apart so the runtime itself is plain C++ and can be
// built into the sanitizer self-test, csrc/tests/runtime_selftest.cpp).  Blocking calls release the GIL.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "runtime.h"

namespace pda_rt {

void bind_runtime(pybind11::module& m) {
  namespace py = pybind11;
  py::class_<StoreServer>(m, "StoreServer")
      .def(py::init<const std::string&, int>(), py::arg("host"), py::arg("port"))
      .def_property_readonly("port", &StoreServer::port)
      .def("stop", &StoreServer::stop);
  py::class_<StoreClient>(m, "StoreClient")
      .def(py::init<const std::string&, int, double>(), py::arg("host"), py::arg("port"), py::arg("timeout"))
      .def("set", &StoreClient::set)
      .def("get", [](StoreClient& c, const std::string& k) {
        std::string v;
        {
          py::gil_scoped_release nogil;
          v = c.get(k);
        }
        return py::bytes(v);
      })
      .def("add", &StoreClient::add)
      .def("check", &StoreClient::check)
      .def("wait", &StoreClient::wait, py::arg("keys"), py::arg("timeout") = 0.0,
           py::call_guard<py::gil_scoped_release>())
      .def("delete_key", &StoreClient::delete_key)
      .def("num_keys", &StoreClient::num_keys)
      .def("compare_set", [](StoreClient& c, const std::string& k, const std::string& e, const std::string& d) {
        return py::bytes(c.compare_set(k, e, d));
      })
      .def("set_timeout", &StoreClient::set_timeout)
      .def_property_readonly("timeout", &StoreClient::timeout);
  py::class_<BucketReducer>(m, "BucketReducer")
      .def(py::init<const std::vector<int64_t>&, const std::vector<int64_t>&, const std::vector<int>&, int64_t,
                    int64_t, int64_t, const std::vector<int64_t>&>(),
           py::arg("numels"), py::arg("elem_sizes"), py::arg("dtype_ids"), py::arg("bucket_cap_bytes"),
           py::arg("first_bucket_bytes"), py::arg("align_elems"), py::arg("order"))
      .def_property_readonly("num_buckets", &BucketReducer::num_buckets)
      .def("bucket_params", &BucketReducer::bucket_params)
      .def("bucket_offsets", &BucketReducer::bucket_offsets)
      .def("bucket_numel", &BucketReducer::bucket_numel)
      .def("bucket_dtype", &BucketReducer::bucket_dtype)
      .def("param_bucket", &BucketReducer::param_bucket)
      .def("prepare", &BucketReducer::prepare)
      .def("mark_ready", &BucketReducer::mark_ready)
      .def("flush_unready", &BucketReducer::flush_unready)
      .def("all_launched", &BucketReducer::all_launched)
      .def("any_marked", &BucketReducer::any_marked)
      .def("unready_params", &BucketReducer::unready_params)
      .def("ready_order", &BucketReducer::ready_order);
  py::class_<HostRing>(m, "HostRing")
      .def(py::init<int, int>())
      .def("listen", &HostRing::listen)
      .def("connect", &HostRing::connect)
      .def("allreduce_f32", &HostRing::allreduce_f32, py::call_guard<py::gil_scoped_release>())
      .def("allreduce_f64", &HostRing::allreduce_f64, py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &HostRing::broadcast, py::call_guard<py::gil_scoped_release>())
      .def("allgather", &HostRing::allgather, py::call_guard<py::gil_scoped_release>())
      .def("barrier", &HostRing::barrier, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("rank", &HostRing::rank)
      .def_property_readonly("world", &HostRing::world);
  py::class_<Watchdog>(m, "Watchdog")
      .def(py::init<double, int, const std::string&, int, double>(), py::arg("timeout"), py::arg("rank"),
           py::arg("action") = "abort", py::arg("exit_code") = 17, py::arg("poll") = 0.5)
      .def("arm", &Watchdog::arm, py::arg("desc"), py::arg("timeout") = -1.0)
      .def("disarm", &Watchdog::disarm)
      .def("attach_stream", &Watchdog::attach_stream, py::arg("ticket"), py::arg("stream"))
      .def_property_readonly("armed", &Watchdog::armed)
      .def("pending", &Watchdog::pending)
      .def("expired", &Watchdog::expired)
      .def_property_readonly("armed_total", &Watchdog::armed_total)
      .def_property_readonly("timeout", &Watchdog::timeout)
      .def("stop", &Watchdog::stop, py::call_guard<py::gil_scoped_release>());
}

}  // namespace pda_rt
