// Native V4L2 capture, see v4l2.h.
#include "v4l2.h"

#include <cerrno>
#include <cstring>
#include <stdexcept>

#include <fcntl.h>
#include <linux/videodev2.h>
#include <poll.h>
#include <sys/ioctl.h>
#include <sys/mman.h>
#include <unistd.h>

namespace ssa {

namespace {

int xioctl(int fd, unsigned long req, void* arg) {
  int r;
  do {
    r = ioctl(fd, req, arg);
  } while (r == -1 && errno == EINTR);
  return r;
}

[[noreturn]] void fail(const std::string& what) {
  throw std::runtime_error("v4l2: " + what + ": " + std::strerror(errno));
}

inline uint8_t sat8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

// BT.601 limited range in 20-bit fixed point (the constants OpenCV's 4:2:x -> RGB
// conversions use): C = Y - 16, D = U - 128, E = V - 128
//   R = 1.164 C + 1.596 E;  G = 1.164 C - 0.391 D - 0.813 E;  B = 1.164 C + 2.018 D
constexpr int kCY = 1220542, kCUB = 2116026, kCUG = -409993, kCVG = -852492, kCVR = 1673527;
constexpr int kShift = 20, kHalf = 1 << (kShift - 1);

inline void px2(int y0, int y1, int u, int v, uint8_t* d) {
  const int du = u - 128, dv = v - 128;
  const int ruv = kHalf + kCVR * dv, guv = kHalf + kCVG * dv + kCUG * du, buv = kHalf + kCUB * du;
  const int c0 = (y0 > 16 ? y0 - 16 : 0) * kCY, c1 = (y1 > 16 ? y1 - 16 : 0) * kCY;
  d[0] = sat8((c0 + buv) >> kShift);
  d[1] = sat8((c0 + guv) >> kShift);
  d[2] = sat8((c0 + ruv) >> kShift);
  d[3] = sat8((c1 + buv) >> kShift);
  d[4] = sat8((c1 + guv) >> kShift);
  d[5] = sat8((c1 + ruv) >> kShift);
}

}  // namespace

void yuv422_to_bgr(const uint8_t* src, int pitch, int W, int H, bool uyvy, uint8_t* dst) {
  if (W % 2) throw std::invalid_argument("yuv422_to_bgr: width must be even");
  const int iy0 = uyvy ? 1 : 0, iu = uyvy ? 0 : 1, iy1 = uyvy ? 3 : 2, iv = uyvy ? 2 : 3;
  for (int y = 0; y < H; ++y) {
    const uint8_t* s = src + (size_t)y * pitch;
    uint8_t* d = dst + (size_t)y * W * 3;
    for (int x = 0; x < W; x += 2, s += 4, d += 6) px2(s[iy0], s[iy1], s[iu], s[iv], d);
  }
}

V4L2Capture::V4L2Capture(const std::string& device, int width, int height, int nbuf) {
  fd_ = ::open(device.c_str(), O_RDWR | O_NONBLOCK);
  if (fd_ < 0) fail("open " + device);
  try {
    v4l2_capability cap{};
    if (xioctl(fd_, VIDIOC_QUERYCAP, &cap) < 0) fail("VIDIOC_QUERYCAP");
    const uint32_t caps = (cap.capabilities & V4L2_CAP_DEVICE_CAPS) ? cap.device_caps : cap.capabilities;
    if (!(caps & V4L2_CAP_VIDEO_CAPTURE)) throw std::runtime_error("v4l2: " + device + " is not a capture device");
    if (!(caps & V4L2_CAP_STREAMING)) throw std::runtime_error("v4l2: " + device + " has no streaming I/O");
    // preferred formats, in order: packed 4:2:2, then 24-bit BGR / RGB
    const uint32_t want[] = {V4L2_PIX_FMT_YUYV, V4L2_PIX_FMT_UYVY, V4L2_PIX_FMT_BGR24, V4L2_PIX_FMT_RGB24};
    bool ok = false;
    for (uint32_t pf : want) {
      v4l2_format f{};
      f.type = V4L2_BUF_TYPE_VIDEO_CAPTURE;
      f.fmt.pix.width = width;
      f.fmt.pix.height = height;
      f.fmt.pix.pixelformat = pf;
      f.fmt.pix.field = V4L2_FIELD_NONE;
      if (xioctl(fd_, VIDIOC_S_FMT, &f) == 0 && f.fmt.pix.pixelformat == pf) {
        fmt_ = pf;
        w_ = (int)f.fmt.pix.width;
        h_ = (int)f.fmt.pix.height;
        const int minpitch = (pf == V4L2_PIX_FMT_BGR24 || pf == V4L2_PIX_FMT_RGB24) ? 3 * w_ : 2 * w_;
        pitch_ = (int)f.fmt.pix.bytesperline >= minpitch ? (int)f.fmt.pix.bytesperline : minpitch;
        ok = true;
        break;
      }
    }
    if (!ok) throw std::runtime_error("v4l2: " + device + " offers none of YUYV/UYVY/BGR24/RGB24");
    v4l2_requestbuffers rb{};
    rb.count = nbuf < 2 ? 2 : nbuf > 16 ? 16 : nbuf;
    rb.type = V4L2_BUF_TYPE_VIDEO_CAPTURE;
    rb.memory = V4L2_MEMORY_MMAP;
    if (xioctl(fd_, VIDIOC_REQBUFS, &rb) < 0) fail("VIDIOC_REQBUFS");
    if (rb.count < 2) throw std::runtime_error("v4l2: driver granted fewer than 2 buffers");
    nbuf_ = rb.count > 16 ? 16 : (int)rb.count;
    for (int i = 0; i < nbuf_; ++i) {
      v4l2_buffer b{};
      b.type = V4L2_BUF_TYPE_VIDEO_CAPTURE;
      b.memory = V4L2_MEMORY_MMAP;
      b.index = i;
      if (xioctl(fd_, VIDIOC_QUERYBUF, &b) < 0) fail("VIDIOC_QUERYBUF");
      void* p = mmap(nullptr, b.length, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, b.m.offset);
      if (p == MAP_FAILED) fail("mmap");
      bufs_[i] = {p, b.length};
      if (xioctl(fd_, VIDIOC_QBUF, &b) < 0) fail("VIDIOC_QBUF");
    }
    v4l2_buf_type t = V4L2_BUF_TYPE_VIDEO_CAPTURE;
    if (xioctl(fd_, VIDIOC_STREAMON, &t) < 0) fail("VIDIOC_STREAMON");
    streaming_ = true;
  } catch (...) {
    close();
    throw;
  }
}

V4L2Capture::~V4L2Capture() { close(); }

std::string V4L2Capture::fourcc() const {
  char s[5] = {(char)(fmt_ & 255), (char)((fmt_ >> 8) & 255), (char)((fmt_ >> 16) & 255), (char)(fmt_ >> 24), 0};
  return s;
}

bool V4L2Capture::read(uint8_t* dst, int timeout_ms, uint32_t* seq, int64_t* ts_us) {
  if (fd_ < 0) return false;
  pollfd pfd{fd_, POLLIN, 0};
  int r;
  do {
    r = poll(&pfd, 1, timeout_ms);
  } while (r < 0 && errno == EINTR);
  if (r <= 0) return false;
  v4l2_buffer b{};
  b.type = V4L2_BUF_TYPE_VIDEO_CAPTURE;
  b.memory = V4L2_MEMORY_MMAP;
  if (xioctl(fd_, VIDIOC_DQBUF, &b) < 0) {
    if (errno == EAGAIN) return false;
    fail("VIDIOC_DQBUF");
  }
  const uint8_t* src = static_cast<const uint8_t*>(bufs_[b.index].p);
  const size_t need = (size_t)pitch_ * (h_ - 1) + (size_t)w_ * (fmt_ == V4L2_PIX_FMT_YUYV || fmt_ == V4L2_PIX_FMT_UYVY ? 2 : 3);
  bool good = b.bytesused == 0 || b.bytesused >= need;  // some drivers leave bytesused 0
  if (good) {
    if (fmt_ == V4L2_PIX_FMT_YUYV || fmt_ == V4L2_PIX_FMT_UYVY) {
      yuv422_to_bgr(src, pitch_, w_, h_, fmt_ == V4L2_PIX_FMT_UYVY, dst);
    } else {
      const bool rgb = fmt_ == V4L2_PIX_FMT_RGB24;
      for (int y = 0; y < h_; ++y) {
        const uint8_t* s = src + (size_t)y * pitch_;
        uint8_t* d = dst + (size_t)y * w_ * 3;
        if (!rgb) {
          std::memcpy(d, s, (size_t)w_ * 3);
        } else {
          for (int x = 0; x < w_; ++x) {
            d[3 * x] = s[3 * x + 2];
            d[3 * x + 1] = s[3 * x + 1];
            d[3 * x + 2] = s[3 * x];
          }
        }
      }
    }
  }
  if (seq) *seq = b.sequence;
  if (ts_us) *ts_us = (int64_t)b.timestamp.tv_sec * 1000000 + b.timestamp.tv_usec;
  if (xioctl(fd_, VIDIOC_QBUF, &b) < 0) fail("VIDIOC_QBUF");
  return good;
}

void V4L2Capture::close() {
  if (fd_ < 0) return;
  if (streaming_) {
    v4l2_buf_type t = V4L2_BUF_TYPE_VIDEO_CAPTURE;
    xioctl(fd_, VIDIOC_STREAMOFF, &t);
    streaming_ = false;
  }
  for (int i = 0; i < nbuf_; ++i)
    if (bufs_[i].p) munmap(bufs_[i].p, bufs_[i].n);
  nbuf_ = 0;
  ::close(fd_);
  fd_ = -1;
}

}  // namespace ssa
