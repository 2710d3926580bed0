// pybind11 bindings of the host-side native pieces (module: _host).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "contours.h"
#include "records.h"
#include "v4l2.h"

namespace py = pybind11;
using namespace ssa;

namespace {

using U8 = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>;
using I32 = py::array_t<int32_t, py::array::c_style | py::array::forcecast>;

std::vector<Pt> to_pts(const I32& a) {
  if (a.ndim() != 2 || a.shape(1) != 2) throw std::invalid_argument("points must be (N, 2) int32");
  std::vector<Pt> p(a.shape(0));
  auto r = a.unchecked<2>();
  for (ssize_t i = 0; i < a.shape(0); ++i) p[i] = {r(i, 0), r(i, 1)};
  return p;
}

py::array_t<int32_t> from_pts(const std::vector<Pt>& p) {
  py::array_t<int32_t> a({(ssize_t)p.size(), (ssize_t)2});
  auto w = a.mutable_unchecked<2>();
  for (size_t i = 0; i < p.size(); ++i) {
    w(i, 0) = p[i].x;
    w(i, 1) = p[i].y;
  }
  return a;
}

py::list find_contours(const U8& mask) {
  if (mask.ndim() != 2) throw std::invalid_argument("mask must be 2-D");
  const int H = (int)mask.shape(0), W = (int)mask.shape(1);
  std::vector<Contour> cs;
  {
    py::gil_scoped_release rel;
    cs = find_contours_tree(mask.data(), H, W, W);
  }
  py::list out;
  for (const Contour& c : cs) {
    py::dict d;
    d["points"] = from_pts(c.simple);
    d["chain"] = from_pts(c.chain);
    d["is_hole"] = c.is_hole;
    d["parent"] = c.parent;
    d["start"] = py::make_tuple(c.start.x, c.start.y);
    out.append(d);
  }
  return out;
}

py::dict moments(const I32& pts) {
  Moments m = contour_moments(to_pts(pts));
  py::dict d;
  d["m00"] = m.m00;
  d["m10"] = m.m10;
  d["m01"] = m.m01;
  d["a00"] = m.a00;
  d["a10"] = m.a10;
  d["a01"] = m.a01;
  return d;
}

py::array_t<uint8_t> fill(const I32& pts, int H, int W) {
  py::array_t<uint8_t> out({(ssize_t)H, (ssize_t)W});
  std::memset(out.mutable_data(), 0, (size_t)H * W);
  fill_contour(to_pts(pts), H, W, out.mutable_data());
  return out;
}

py::array_t<uint8_t> mask(const U8& labels, const I32& palette, int thr) {
  if (labels.ndim() != 2) throw std::invalid_argument("labels must be 2-D");
  if (palette.size() != 256 * 3) throw std::invalid_argument("palette must be (256, 3)");
  const int h = (int)labels.shape(0), w = (int)labels.shape(1);
  py::array_t<uint8_t> out({(ssize_t)h, (ssize_t)w});
  palette_mask(labels.data(), h, w, w, palette.data(), thr, out.mutable_data());
  return out;
}

py::list segments(const U8& labels, const I32& palette, double min_area) {
  if (labels.ndim() != 2) throw std::invalid_argument("labels must be 2-D");
  if (palette.size() != 256 * 3) throw std::invalid_argument("palette must be (256, 3)");
  const int h = (int)labels.shape(0), w = (int)labels.shape(1);
  std::vector<Segment> segs;
  {
    py::gil_scoped_release rel;
    segs = segments_exact(labels.data(), h, w, w, palette.data(), min_area, 256);
  }
  py::list out;
  for (const Segment& s : segs)
    out.append(py::make_tuple(s.label, s.score, s.area, s.cx, s.cy, s.contour, s.is_hole));
  return out;
}

}  // namespace

PYBIND11_MODULE(_host, m) {
  m.doc() = "Host-side exact contour analysis (Suzuki-Abe border following, OpenCV-equivalent).";
  m.def(
      "unpack_records",
      [](py::array packed, int K, py::array meta, py::array out) {
        // packed: float32 (F, >= 1 + 5K) C-contiguous rows; meta: float64 (F, 3); out: a
        // writable C-contiguous RECORD_DTYPE (40-byte) array of >= F * K rows
        if (packed.ndim() != 2 || packed.dtype().kind() != 'f' || packed.itemsize() != 4 ||
            !(packed.flags() & py::array::c_style) || packed.shape(1) < 1 + 5 * (ssize_t)K)
          throw std::invalid_argument("unpack_records: packed must be C-contiguous float32 (F, 1 + 5K)");
        const ssize_t F = packed.shape(0);
        if (meta.ndim() != 2 || meta.shape(0) != F || meta.shape(1) != 3 || meta.itemsize() != 8 ||
            meta.dtype().kind() != 'f' || !(meta.flags() & py::array::c_style))
          throw std::invalid_argument("unpack_records: meta must be C-contiguous float64 (F, 3)");
        if (out.ndim() != 1 || out.itemsize() != (ssize_t)sizeof(Record) || !out.writeable() ||
            !(out.flags() & py::array::c_style) || out.shape(0) < F * K)
          throw std::invalid_argument("unpack_records: out must be a writable RECORD_DTYPE array of F * K rows");
        const UnpackStats st = unpack_records(static_cast<const float*>(packed.data()), F, K, packed.shape(1),
                                              static_cast<const double*>(meta.data()),
                                              static_cast<Record*>(out.mutable_data()), out.shape(0));
        return py::make_tuple(st.records, st.overflow, st.pool_lost);
      },
      py::arg("packed"), py::arg("K"), py::arg("meta"), py::arg("out"),
      "Packed per-frame device records -> RECORD_DTYPE rows in push order; returns (rows, "
      "overflow frames, pool-exhausted frames)");
  m.def("find_contours", &find_contours, py::arg("mask"),
        "findContours(RETR_TREE, CHAIN_APPROX_SIMPLE) on a 0/nonzero uint8 mask.");
  m.def("contour_area", [](const I32& p) { return contour_area(to_pts(p)); });
  m.def("moments", &moments);
  m.def("fill", &fill, py::arg("points"), py::arg("H"), py::arg("W"));
  m.def("palette_mask", &mask, py::arg("labels"), py::arg("palette"), py::arg("thr") = 127);
  m.def("segments", &segments, py::arg("labels"), py::arg("palette"), py::arg("min_area"),
        "Reference post-processing of one cropped label map -> "
        "[(label, score, area, cx, cy, contour_index, is_hole)] in contour order.");

  m.def("yuv422_to_bgr", [](const U8& src, bool uyvy) {
    if (src.ndim() != 2 || src.shape(1) % 4) throw std::invalid_argument("yuv422_to_bgr: (H, 2*W) uint8, W even");
    const int H = (int)src.shape(0), W = (int)src.shape(1) / 2;
    py::array_t<uint8_t> out({(ssize_t)H, (ssize_t)W, (ssize_t)3});
    yuv422_to_bgr(src.data(), 2 * W, W, H, uyvy, out.mutable_data());
    return out;
  }, py::arg("src"), py::arg("uyvy") = false,
        "Packed 4:2:2 (YUYV, or UYVY) -> BGR, BT.601 limited range (OpenCV's COLOR_YUV2BGR_YUYV convention).");

  py::class_<V4L2Capture>(m, "V4L2Capture")
      .def(py::init<const std::string&, int, int, int>(), py::arg("device"), py::arg("width") = 640,
           py::arg("height") = 480, py::arg("nbuf") = 4)
      .def_property_readonly("width", &V4L2Capture::width)
      .def_property_readonly("height", &V4L2Capture::height)
      .def_property_readonly("fourcc", &V4L2Capture::fourcc)
      .def("read_into", [](V4L2Capture& c, py::array_t<uint8_t, py::array::c_style> dst, int timeout_ms) {
             if (dst.ndim() != 3 || dst.shape(0) != c.height() || dst.shape(1) != c.width() || dst.shape(2) != 3)
               throw std::invalid_argument("read_into: dst must be (height, width, 3) uint8");
             uint32_t seq = 0;
             int64_t ts = 0;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = c.read(dst.mutable_data(), timeout_ms, &seq, &ts);
             }
             return py::make_tuple(ok, seq, ts);
           }, py::arg("dst"), py::arg("timeout_ms") = 1000,
           "Next frame as BGR into dst; returns (ok, driver sequence, timestamp us).")
      .def("close", &V4L2Capture::close);
}
