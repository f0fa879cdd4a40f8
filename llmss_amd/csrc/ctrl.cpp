// Python binding of the shared-memory control ring (csrc/ctrl_ring.h: protocol, shm lifetime, back-off) into
// module llmss_amd._C. Every blocking call (send / recv / wait_attached) runs with the GIL released; recv() turns
// the message into Python bytes after re-acquiring it. Timeouts surface as TimeoutError.
#include <pybind11/pybind11.h>

#include "ctrl_ring.h"

namespace py = pybind11;
using llmss_ctrl::CtrlRing;

void register_ctrl(py::module_& m) {
  py::register_exception<llmss_ctrl::Timeout>(m, "CtrlRingTimeout", PyExc_TimeoutError);
  py::class_<CtrlRing>(m, "CtrlRing")
      .def(py::init<const std::string&, bool, int64_t, int, int>(), py::arg("name"), py::arg("create"),
           py::arg("capacity") = 1 << 24, py::arg("nreaders") = 1, py::arg("reader") = 0)
      .def("wait_attached", &CtrlRing::wait_attached, py::call_guard<py::gil_scoped_release>())
      .def(
          "send",
          [](CtrlRing& r, const std::string& msg, double timeout_s) {
            py::gil_scoped_release nogil;
            r.send(msg, timeout_s);
          },
          py::arg("msg"), py::arg("timeout_s") = -1.0)
      .def(
          "recv",
          [](CtrlRing& r, double timeout_s) {
            std::string s;
            {
              py::gil_scoped_release nogil;
              s = r.recv(timeout_s);
            }
            return py::bytes(s);
          },
          py::arg("timeout_s") = -1.0)
      .def("close_producer", &CtrlRing::close_producer)
      .def("unlink", &CtrlRing::unlink)
      .def_property_readonly("capacity", &CtrlRing::capacity)
      .def_property_readonly("nreaders", &CtrlRing::nreaders)
      .def_property_readonly("attached", &CtrlRing::attached);
}
