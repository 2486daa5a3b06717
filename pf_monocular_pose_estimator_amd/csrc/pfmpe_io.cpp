// pfmpe_io.cpp — the engine's configuration and recorded-stream boundary, host C++.
//
//   * marker YAML      README.md:95-117, pf_mpe/marker_positions/*.yaml, read by the node through
//                      nh_private_.getParam("marker_positions") (pf_mpe/src/monocular_pose_estimator.cpp:81-126)
//   * launch params    <param name="..." value="..."/> of pf_mpe/launch/*.launch, the names
//                      dynamicParametersCallback copies into PoseEstimator (monocular_pose_estimator.cpp:479-527)
//   * camera_info      the sensor_msgs/CameraInfo echo of README.md:127-143 (K, D, width, height)
//   * blob streams     a compact binary record of per-frame undistorted detections (image_points_,
//                      led_detector.cpp:192-212 -> PE:469), so a multi-GPU harness can replay recorded
//                      detections straight into the device blob bank (pfmpe_stage_blob_bank)
// No YAML/XML library: the formats above are line-oriented and parsed by hand.
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pfmpe.h"

namespace {

std::string trim(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && std::isspace((unsigned char)s[a])) ++a;
  while (b > a && std::isspace((unsigned char)s[b - 1])) --b;
  return s.substr(a, b - a);
}
std::string strip_comment(const std::string& s) {
  const size_t h = s.find('#');
  return h == std::string::npos ? s : s.substr(0, h);
}
std::vector<std::string> lines_of(const char* text) {
  std::vector<std::string> out;
  std::string cur;
  for (const char* p = text; *p; ++p) {
    if (*p == '\n') {
      out.push_back(cur);
      cur.clear();
    } else if (*p != '\r') {
      cur.push_back(*p);
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}
size_t indent_of(const std::string& s) {
  size_t i = 0;
  while (i < s.size() && (s[i] == ' ' || s[i] == '\t')) ++i;
  return i;
}
bool parse_double(const std::string& s, double* v) {
  const std::string t = trim(s);
  if (t.empty()) return false;
  char* end = nullptr;
  const double x = std::strtod(t.c_str(), &end);
  if (end == t.c_str() || !trim(std::string(end)).empty()) return false;
  *v = x;
  return true;
}
// "key: value" pieces of one YAML mapping line (block style) or flow map "{x: 1, y: 2}"
void map_entries(const std::string& body, std::vector<std::pair<std::string, std::string>>& kv) {
  std::string b = trim(body);
  if (!b.empty() && b.front() == '{') {
    const size_t e = b.rfind('}');
    b = b.substr(1, (e == std::string::npos ? b.size() : e) - 1);
    size_t start = 0;
    while (start <= b.size()) {
      size_t comma = b.find(',', start);
      if (comma == std::string::npos) comma = b.size();
      const std::string part = b.substr(start, comma - start);
      const size_t c = part.find(':');
      if (c != std::string::npos) kv.emplace_back(trim(part.substr(0, c)), trim(part.substr(c + 1)));
      start = comma + 1;
    }
    return;
  }
  const size_t c = b.find(':');
  if (c != std::string::npos) kv.emplace_back(trim(b.substr(0, c)), trim(b.substr(c + 1)));
}
// "[a, b, c]" -> numbers
int parse_list(const std::string& s, double* out, int max_n) {
  const size_t a = s.find('['), b = s.rfind(']');
  if (a == std::string::npos || b == std::string::npos || b < a) return -1;
  const std::string in = s.substr(a + 1, b - a - 1);
  int n = 0;
  size_t start = 0;
  while (start <= in.size() && n <= max_n) {
    size_t comma = in.find(',', start);
    if (comma == std::string::npos) comma = in.size();
    double v;
    const std::string item = trim(in.substr(start, comma - start));
    if (!item.empty()) {
      if (!parse_double(item, &v)) return -1;
      if (n < max_n) out[n] = v;
      ++n;
    }
    start = comma + 1;
  }
  return n;
}
bool parse_bool(const std::string& s, bool* v) {
  std::string t = trim(s);
  for (auto& ch : t) ch = (char)std::tolower((unsigned char)ch);
  if (t == "true" || t == "1") {
    *v = true;
    return true;
  }
  if (t == "false" || t == "0") {
    *v = false;
    return true;
  }
  return false;
}
// value of attribute `name` in an XML tag body
bool xml_attr(const std::string& tag, const char* name, std::string* out) {
  size_t p = 0;
  const size_t nl = std::strlen(name);
  while ((p = tag.find(name, p)) != std::string::npos) {
    const bool word_start = p == 0 || std::isspace((unsigned char)tag[p - 1]);
    size_t q = p + nl;
    while (q < tag.size() && std::isspace((unsigned char)tag[q])) ++q;
    if (word_start && q < tag.size() && tag[q] == '=') {
      ++q;
      while (q < tag.size() && std::isspace((unsigned char)tag[q])) ++q;
      if (q < tag.size() && (tag[q] == '"' || tag[q] == '\'')) {
        const char quote = tag[q];
        const size_t e = tag.find(quote, q + 1);
        if (e == std::string::npos) return false;
        *out = trim(tag.substr(q + 1, e - q - 1));
        return true;
      }
    }
    p += nl;
  }
  return false;
}

constexpr char kMagic[4] = {'P', 'F', 'M', 'B'};
constexpr uint32_t kVersion = 1;

}  // namespace

extern "C" {

int pfmpe_parse_marker_yaml(const char* text, double* xyz, int max_markers) {
  if (!text || (!xyz && max_markers > 0) || max_markers < 0) return PFMPE_E_ARG;
  const std::vector<std::string> ls = lines_of(text);
  size_t i = 0;
  for (; i < ls.size(); ++i) {
    const std::string t = trim(strip_comment(ls[i]));
    if (t.rfind("marker_positions", 0) == 0 && t.find(':') != std::string::npos) break;
  }
  if (i == ls.size()) return PFMPE_E_ARG;
  const size_t key_indent = indent_of(ls[i]);
  int n = 0;
  double cur[3] = {0, 0, 0};
  int have = 0;  // bit mask x/y/z of the current item
  bool open = false;
  auto flush = [&]() -> bool {
    if (!open) return true;
    if (have != 7) return false;
    if (n < max_markers)
      for (int k = 0; k < 3; ++k) xyz[3 * n + k] = cur[k];
    ++n;
    open = false;
    have = 0;
    return true;
  };
  for (++i; i < ls.size(); ++i) {
    const std::string raw = strip_comment(ls[i]);
    const std::string t = trim(raw);
    if (t.empty()) continue;
    if (indent_of(raw) <= key_indent && t[0] != '-') break;  // next top-level key
    std::string body = t;
    if (t[0] == '-') {
      if (!flush()) return PFMPE_E_ARG;
      open = true;
      body = t.substr(1);
    }
    std::vector<std::pair<std::string, std::string>> kv;
    map_entries(body, kv);
    for (auto& e : kv) {
      const int k = e.first == "x" ? 0 : e.first == "y" ? 1 : e.first == "z" ? 2 : -1;
      double v;
      if (k < 0 || !open || !parse_double(e.second, &v)) return PFMPE_E_ARG;
      cur[k] = v;
      have |= 1 << k;
    }
  }
  if (!flush()) return PFMPE_E_ARG;
  return n;
}

void pfmpe_default_launch_config(pfmpe_launch_config* cfg) {
  if (!cfg) return;
  std::memset(cfg, 0, sizeof(*cfg));
  pfmpe_default_params(&cfg->pf);
  pfmpe_default_init_params(&cfg->init);
  cfg->num_objects = 1;
  cfg->use_particle_filter = 1;
}

int pfmpe_parse_launch(const char* text, pfmpe_launch_config* cfg) {
  if (!text || !cfg) return PFMPE_E_ARG;
  std::string all(text);
  // drop <!-- comments -->
  for (size_t a; (a = all.find("<!--")) != std::string::npos;) {
    const size_t b = all.find("-->", a);
    all.erase(a, b == std::string::npos ? std::string::npos : b + 3 - a);
  }
  int known = 0;
  size_t p = 0;
  while ((p = all.find("<param", p)) != std::string::npos) {
    const size_t e = all.find('>', p);
    if (e == std::string::npos) break;
    const std::string tag = all.substr(p + 6, e - p - 6);
    p = e;
    std::string name, value;
    if (!xml_attr(tag, "name", &name) || !xml_attr(tag, "value", &value)) continue;
    double v = 0;
    bool b = false;
    const bool num = parse_double(value, &v);
    const bool isb = parse_bool(value, &b);
    int hit = 1;
    if (name == "back_projection_pixel_tolerance" && num) cfg->pf.tol = v;
    else if (name == "back_projection_pixel_tolerance_PF" && num) cfg->pf.tol_pf = v;
    else if (name == "maxAngularNoise" && num) cfg->pf.ang_max = v;
    else if (name == "minAngularNoise" && num) cfg->pf.ang_min = v;
    else if (name == "maxTransitionNoise" && num) cfg->pf.trans_max = v;
    else if (name == "minTransitionNoise" && num) cfg->pf.trans_min = v;
    else if (name == "certainty_threshold" && num) cfg->init.certainty_threshold = v;
    else if (name == "valid_correspondence_threshold" && num) cfg->init.valid_corr_threshold = v;
    else if (name == "N_Particle" && num) cfg->init.n_particles = (int32_t)v;
    else if (name == "numUAV" && num) cfg->num_objects = (int32_t)v;
    else if (name.rfind("numberOfMarkersUAV", 0) == 0 && name.size() == 19 && name[18] >= '1' && name[18] <= '4' && num)
      cfg->markers_per_object[name[18] - '1'] = (int32_t)v;
    else if (name.rfind("bMarkerNr", 0) == 0 && name.size() == 10 && name[9] >= '1' && name[9] <= '5' && isb)
      cfg->downgrade[name[9] - '1'] = b ? 1 : 0;
    else if (name == "bUseParticleFilter" && isb) cfg->use_particle_filter = b ? 1 : 0;
    else hit = 0;
    known += hit;
  }
  return known;
}

int pfmpe_parse_camera_info(const char* text, double* K, double* D, int32_t* width, int32_t* height) {
  if (!text) return PFMPE_E_ARG;
  int found = 0;
  for (const std::string& raw : lines_of(text)) {
    const std::string t = trim(strip_comment(raw));
    const size_t c = t.find(':');
    if (c == std::string::npos) continue;
    const std::string key = trim(t.substr(0, c)), val = trim(t.substr(c + 1));
    double tmp[16];
    double v;
    if (key == "K" && K) {
      if (parse_list(val, tmp, 9) != 9) return PFMPE_E_ARG;
      std::memcpy(K, tmp, 9 * sizeof(double));
      found |= 1;
    } else if (key == "D" && D) {
      const int n = parse_list(val, tmp, 16);
      if (n < 0) return PFMPE_E_ARG;
      for (int k = 0; k < 5; ++k) D[k] = k < n ? tmp[k] : 0.0;  // plumb_bob k1 k2 p1 p2 k3
      found |= 2;
    } else if (key == "width" && width && parse_double(val, &v)) {
      *width = (int32_t)v;
      found |= 4;
    } else if (key == "height" && height && parse_double(val, &v)) {
      *height = (int32_t)v;
      found |= 8;
    }
  }
  return found;
}

int pfmpe_write_blob_stream(const char* path, const double* timestamps, const double* blobs, const int32_t* offsets,
                            int n_frames) {
  if (!path || !offsets || n_frames < 0) return PFMPE_E_ARG;
  for (int f = 0; f < n_frames; ++f)
    if (offsets[f + 1] < offsets[f] || offsets[f] < 0) return PFMPE_E_ARG;
  if (n_frames > 0 && offsets[n_frames] > 0 && !blobs) return PFMPE_E_ARG;
  FILE* fp = std::fopen(path, "wb");
  if (!fp) return PFMPE_E_ARG;
  const uint32_t hdr[3] = {kVersion, (uint32_t)n_frames, 0};
  bool ok = std::fwrite(kMagic, 1, 4, fp) == 4 && std::fwrite(hdr, 4, 3, fp) == 3;
  for (int f = 0; f < n_frames && ok; ++f) {
    const double ts = timestamps ? timestamps[f] : 0.0;
    const uint32_t fh[2] = {(uint32_t)(offsets[f + 1] - offsets[f]), 0};
    ok = std::fwrite(&ts, 8, 1, fp) == 1 && std::fwrite(fh, 4, 2, fp) == 2;
    if (ok && fh[0]) ok = std::fwrite(blobs + 2 * (size_t)offsets[f], 16, fh[0], fp) == fh[0];
  }
  ok = (std::fclose(fp) == 0) && ok;
  return ok ? PFMPE_OK : PFMPE_E_ARG;
}

int pfmpe_read_blob_stream(const char* path, double* timestamps, double* blobs, int32_t* offsets, int max_frames,
                           int64_t max_blobs, int* n_frames, int64_t* n_blobs) {
  if (!path || !n_frames || !n_blobs) return PFMPE_E_ARG;
  FILE* fp = std::fopen(path, "rb");
  if (!fp) return PFMPE_E_ARG;
  char magic[4];
  uint32_t hdr[3];
  if (std::fread(magic, 1, 4, fp) != 4 || std::memcmp(magic, kMagic, 4) != 0 || std::fread(hdr, 4, 3, fp) != 3 ||
      hdr[0] != kVersion) {
    std::fclose(fp);
    return PFMPE_E_ARG;
  }
  const int nf = (int)hdr[1];
  int64_t total = 0;
  int rc = PFMPE_OK;
  if (offsets && max_frames >= nf) offsets[0] = 0;
  for (int f = 0; f < nf; ++f) {
    double ts;
    uint32_t fh[2];
    if (std::fread(&ts, 8, 1, fp) != 1 || std::fread(fh, 4, 2, fp) != 2 || fh[0] > PFMPE_MAX_BLOBS) {
      rc = PFMPE_E_ARG;
      break;
    }
    const bool store = blobs && offsets && timestamps && f < max_frames && total + fh[0] <= max_blobs;
    if (store) {
      timestamps[f] = ts;
      if (fh[0] && std::fread(blobs + 2 * total, 16, fh[0], fp) != fh[0]) {
        rc = PFMPE_E_ARG;
        break;
      }
    } else if (fh[0] && std::fseek(fp, 16L * fh[0], SEEK_CUR) != 0) {
      rc = PFMPE_E_ARG;
      break;
    }
    total += fh[0];
    if (offsets && f < max_frames) offsets[f + 1] = (int32_t)total;
  }
  std::fclose(fp);
  *n_frames = nf;
  *n_blobs = total;
  if (rc == PFMPE_OK && (blobs || offsets || timestamps) && (max_frames < nf || max_blobs < total)) return PFMPE_E_CAP;
  return rc;
}

int pfmpe_stage_blob_stream(pfmpe_ctx* ctx, const char* path, int* n_frames) {
  if (!ctx || !path) return PFMPE_E_ARG;
  int nf = 0;
  int64_t nb = 0;
  int rc = pfmpe_read_blob_stream(path, nullptr, nullptr, nullptr, 0, 0, &nf, &nb);
  if (rc != PFMPE_OK) return rc;
  if (nf < 1) return PFMPE_E_ARG;
  std::vector<double> ts(nf), bl(2 * (size_t)std::max<int64_t>(nb, 1));
  std::vector<int32_t> off(nf + 1);
  rc = pfmpe_read_blob_stream(path, ts.data(), bl.data(), off.data(), nf, nb, &nf, &nb);
  if (rc != PFMPE_OK) return rc;
  if (n_frames) *n_frames = nf;
  return pfmpe_stage_blob_bank(ctx, bl.data(), off.data(), nf);
}

}  // extern "C"
