// offline_log.cc -- see offline_log.h.
#include "offline_log.h"

#include <zlib.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <stdexcept>

namespace disinfect {

std::vector<LogEntry> parse_log_entries(const std::string& logdir, const SE3<float>& extrinsics) {
  std::vector<LogEntry> out;
  std::ifstream fin(logdir + "/trajectory.txt");
  int id;
  float m[12];
  while (fin >> id >> m[0] >> m[1] >> m[2] >> m[3] >> m[4] >> m[5] >> m[6] >> m[7] >> m[8] >> m[9] >>
         m[10] >> m[11])
    out.push_back({id, extrinsics * SE3<float>::FromMatrix(m, 4)});
  return out;
}

namespace {

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

int paeth(int a, int b, int c) {
  const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  if (pa <= pb && pa <= pc) return a;
  return pb <= pc ? b : c;
}

}  // namespace

Mat read_png(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return Mat();
  std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (buf.size() < 8 || std::memcmp(buf.data(), sig, 8) != 0) throw std::runtime_error(path + ": not a PNG");
  uint32_t W = 0, H = 0;
  int depth = 0, ctype = -1;
  std::vector<uint8_t> idat;
  for (size_t p = 8; p + 12 <= buf.size();) {
    const uint32_t len = be32(&buf[p]);
    if (p + 12 + (size_t)len > buf.size()) throw std::runtime_error(path + ": truncated chunk");
    const std::string type(reinterpret_cast<const char*>(&buf[p + 4]), 4);
    const uint8_t* d = &buf[p + 8];
    if (type == "IHDR") {
      W = be32(d);
      H = be32(d + 4);
      depth = d[8];
      ctype = d[9];
      if (d[12] != 0) throw std::runtime_error(path + ": interlaced PNG not supported");
    } else if (type == "IDAT") {
      idat.insert(idat.end(), d, d + len);
    } else if (type == "IEND") {
      break;
    }
    p += 12 + len;
  }
  const int chans = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 6 ? 4 : 0;
  if (!W || !H || !chans || (depth != 8 && depth != 16))
    throw std::runtime_error(path + ": unsupported PNG (grey / RGB / RGBA, 8 or 16 bit)");
  const size_t bpp = (size_t)chans * depth / 8, stride = (size_t)W * bpp;
  std::vector<uint8_t> raw(H * (stride + 1));
  uLongf n = (uLongf)raw.size();
  if (uncompress(raw.data(), &n, idat.data(), (uLong)idat.size()) != Z_OK || n != raw.size())
    throw std::runtime_error(path + ": bad zlib stream");
  std::vector<uint8_t> img(H * stride);
  for (uint32_t y = 0; y < H; ++y) {  // undo the scanline filters (PNG spec 9.2)
    const uint8_t ft = raw[y * (stride + 1)];
    const uint8_t* s = &raw[y * (stride + 1) + 1];
    uint8_t* o = &img[y * stride];
    const uint8_t* up = y ? &img[(y - 1) * stride] : nullptr;
    for (size_t i = 0; i < stride; ++i) {
      const int a = i >= bpp ? o[i - bpp] : 0, b = up ? up[i] : 0, c = (up && i >= bpp) ? up[i - bpp] : 0;
      int v = s[i];
      switch (ft) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) >> 1; break;
        case 4: v += paeth(a, b, c); break;
        default: throw std::runtime_error(path + ": bad filter type");
      }
      o[i] = (uint8_t)v;
    }
  }
  if (chans == 1) {
    Mat m((int)H, (int)W, depth == 8 ? CV_8UC1 : CV_16UC1);
    if (depth == 8) {
      std::memcpy(m.data, img.data(), img.size());
    } else {  // big-endian samples
      uint16_t* q = m.ptr<uint16_t>();
      for (size_t i = 0; i < (size_t)W * H; ++i) q[i] = (uint16_t)(img[2 * i] << 8 | img[2 * i + 1]);
    }
    return m;
  }
  Mat m((int)H, (int)W, CV_8UC3);  // imread(IMREAD_COLOR) + cvtColor(BGR2RGB) == the file's RGB
  uint8_t* q = m.data;
  const size_t step = depth / 8;
  for (size_t i = 0; i < (size_t)W * H; ++i)
    for (int c = 0; c < 3; ++c) q[3 * i + c] = img[i * bpp + c * step];  // 16-bit: high byte
  return m;
}

void get_images_by_id(int id, float depth_scale, Mat* img_rgb, Mat* img_depth, Mat* img_ht,
                      Mat* img_lt, const std::string& logdir) {
  const std::string base = logdir + "/" + std::to_string(id);
  *img_rgb = read_png(base + "_rgb.png");
  const Mat d = read_png(base + "_depth.png");
  const Mat h = read_png(base + "_ht.png");
  const Mat l = read_png(base + "_no_ht.png");
  if (img_rgb->empty() || d.empty()) throw std::runtime_error(base + ": missing rgb / depth frame");
  auto to_float = [](const Mat& src, float alpha) {  // convertTo(CV_32FC1, alpha)
    Mat out(src.rows, src.cols, CV_32FC1);
    float* o = out.ptr<float>();
    for (size_t i = 0; i < src.total(); ++i)
      o[i] = (float)(src.type() == CV_16UC1 ? src.ptr<uint16_t>()[i] : src.data[i]) * alpha;
    return out;
  };
  *img_depth = to_float(d, (float)(1. / depth_scale));
  if (!h.empty() && !l.empty()) {
    *img_ht = to_float(h, (float)(1. / 65535));
    *img_lt = to_float(l, (float)(1. / 65535));
  } else {  // offline.cc:80-81
    *img_ht = Mat(d.rows, d.cols, CV_32FC1);
    std::memset(img_ht->data, 0, img_ht->total() * 4);
    *img_lt = Mat::ones(d.rows, d.cols, CV_32FC1);
  }
}

}  // namespace disinfect
