// Native V4L2 camera capture (frame source of the producer loop without OpenCV).
//
// The reference reads frames with cv2.VideoCapture(camera_idx) (sem_seg_server.py:144-148,
// 268-270): a V4L2 device on the Coral board, converted to BGR by OpenCV. OpenCV is not
// part of this image, so this is the capture path itself: open /dev/videoN, negotiate a
// packed 4:2:2 (YUYV / UYVY) or 24-bit BGR/RGB format, mmap-streaming I/O with a small
// driver-side ring, and a fixed-point YUV -> BGR conversion straight into the caller's
// (pinned) frame buffer. Conversion follows OpenCV's COLOR_YUV2BGR_YUYV convention
// (BT.601 limited range, 20-bit fixed point); parity with OpenCV itself is unpinned
// (cv2 not importable), tests check it against the float formula.
#pragma once
#include <cstdint>
#include <string>

namespace ssa {

// YUYV (Y0 U Y1 V) / UYVY (U Y0 V Y1) -> BGR, one row pitch `pitch` bytes.
void yuv422_to_bgr(const uint8_t* src, int pitch, int W, int H, bool uyvy, uint8_t* dst);

class V4L2Capture {
 public:
  // Opens `device`, asks for width x height (the driver may pick another size; see
  // width()/height()), nbuf mmap buffers. Throws std::runtime_error on failure.
  V4L2Capture(const std::string& device, int width, int height, int nbuf = 4);
  ~V4L2Capture();
  V4L2Capture(const V4L2Capture&) = delete;
  V4L2Capture& operator=(const V4L2Capture&) = delete;

  int width() const { return w_; }
  int height() const { return h_; }
  std::string fourcc() const;
  // Dequeues the next frame (waits at most timeout_ms), converts it to BGR into dst
  // (height x width x 3) and re-queues the buffer. Returns false on timeout / EOF.
  // seq / ts_us: driver sequence number and capture timestamp (microseconds).
  bool read(uint8_t* dst, int timeout_ms, uint32_t* seq, int64_t* ts_us);
  void close();

 private:
  int fd_ = -1;
  int w_ = 0, h_ = 0, pitch_ = 0;
  uint32_t fmt_ = 0;
  struct Buf { void* p; size_t n; };
  Buf bufs_[16] = {};
  int nbuf_ = 0;
  bool streaming_ = false;
};

}  // namespace ssa
