// Torch-free core of the native text pipeline (text_pipeline.cpp): HTML-tag stripping, BERT
// BasicTokenizer, WordPiece and the fixed-length row encoder.  Header-only so the same code is
// compiled into the extension and into the host sanitizer harness (tests/native/text_core_check.cpp,
// built with -fsanitize=address,undefined by tests/test_native_sanitizers_cpu.py).
#pragma once

#include <algorithm>
#include <cctype>
#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

namespace pcmp_rt {

inline bool is_ws(unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
inline bool is_punct(unsigned char c) {
  return (c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126);
}

// strip HTML tags: every '<...>' span becomes a single space (regex '<[^>]+>' semantics)
inline std::string strip_tags(const std::string& s) {
  std::string out;
  out.reserve(s.size());
  size_t i = 0;
  while (i < s.size()) {
    if (s[i] == '<') {
      size_t j = s.find('>', i + 1);
      if (j != std::string::npos && j > i + 1) {
        out.push_back(' ');
        i = j + 1;
        continue;
      }
    }
    out.push_back(s[i++]);
  }
  return out;
}

// BERT BasicTokenizer (ASCII punctuation split; bytes >= 0x80 kept inside words)
inline void basic_tokenize(const std::string& text, bool lower, std::vector<std::string>& toks) {
  std::string cur;
  for (unsigned char c : text) {
    if (c == 0 || c == 0xfd) continue;
    if (is_ws(c)) {
      if (!cur.empty()) { toks.push_back(cur); cur.clear(); }
    } else if (is_punct(c)) {
      if (!cur.empty()) { toks.push_back(cur); cur.clear(); }
      toks.emplace_back(1, (char)c);
    } else {
      cur.push_back(lower && c < 128 ? (char)std::tolower(c) : (char)c);
    }
  }
  if (!cur.empty()) toks.push_back(cur);
}

struct Vocab {
  std::unordered_map<std::string, int64_t> map;
  int64_t unk = 100, cls = 101, sep = 102;
};

inline void wordpiece(const std::string& w, const Vocab& v, std::vector<int64_t>& out) {
  if (w.size() > 100) { out.push_back(v.unk); return; }
  std::vector<int64_t> pieces;
  size_t start = 0;
  while (start < w.size()) {
    size_t end = w.size();
    int64_t found = -1;
    while (start < end) {
      std::string sub = w.substr(start, end - start);
      if (start > 0) sub = "##" + sub;
      auto it = v.map.find(sub);
      if (it != v.map.end()) { found = it->second; break; }
      --end;
    }
    if (found < 0) { out.push_back(v.unk); return; }
    pieces.push_back(found);
    start = end;
  }
  out.insert(out.end(), pieces.begin(), pieces.end());
}

// one review -> [CLS] wordpieces... [SEP] truncated (post) into row[0..max_len), zero padding (post);
// mask[i] = row[i] > 0.  max_len >= 2.
inline void encode_row(const std::string& text, const Vocab& v, int64_t max_len, bool lower, bool strip,
                       int64_t* row, int64_t* mask) {
  std::vector<std::string> toks;
  basic_tokenize(strip ? strip_tags(text) : text, lower, toks);
  std::vector<int64_t> wp;
  wp.reserve(toks.size() + 4);
  for (const auto& t : toks) {
    wordpiece(t, v, wp);
    if ((int64_t)wp.size() >= max_len) break;
  }
  const int64_t body = std::min<int64_t>((int64_t)wp.size(), max_len - 2);
  int64_t k = 0;
  row[k++] = v.cls;
  for (int64_t i = 0; i < body; ++i) row[k++] = wp[i];
  row[k++] = v.sep;
  for (; k < max_len; ++k) row[k] = 0;
  for (int64_t i = 0; i < max_len; ++i) mask[i] = row[i] > 0 ? 1 : 0;
}

}  // namespace pcmp_rt
