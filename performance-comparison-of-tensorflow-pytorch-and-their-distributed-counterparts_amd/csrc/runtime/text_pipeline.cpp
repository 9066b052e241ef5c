// Native text pre-processing pipeline (host C++, OpenMP) for the IMDB classifier path.
//
// Replaces, in one multithreaded pass over all reviews, the reference's Python-loop pipeline
// (pytorch_on_language_distr.py:34-103):
//   rm_tags (regex '<[^>]+>' -> ' ')  ->  BertTokenizer(do_lower_case=True).encode(
//   add_special_tokens=True, max_length=128) (BasicTokenizer: lower-case, whitespace +
//   punctuation split; WordPiece greedy longest-match-first with '##' continuations,
//   100-char word limit -> [UNK]) -> pad_sequences(maxlen=128, padding='post',
//   truncating='post', value=0) -> attention_mask = int(token_id > 0).
// The reference tokenises every review in a single-threaded Python loop on every rank; here each
// rank runs it once at native speed across all cores.
//
// Exposed as torch.ops.pcmp.text_encode(str[] texts, str[] vocab, int max_len, bool lower,
// bool strip_tags) -> [ids int64 [N,max_len], mask int64 [N,max_len]] and
// torch.ops.pcmp.text_basic_tokenize(str[] texts, bool lower, bool strip_tags) -> str[] (space-
// joined basic tokens, used to build a vocabulary when no vocab file is available offline).
#include <torch/extension.h>

#include <string>
#include <unordered_map>
#include <vector>

namespace pcmp_rt {

static inline bool is_ws(unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
static inline bool is_punct(unsigned char c) {
  return (c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126);
}

// strip HTML tags: every '<...>' span becomes a single space (regex '<[^>]+>' semantics)
static std::string strip_tags(const std::string& s) {
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
static void basic_tokenize(const std::string& text, bool lower, std::vector<std::string>& toks) {
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

static void wordpiece(const std::string& w, const Vocab& v, std::vector<int64_t>& out) {
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

std::vector<at::Tensor> text_encode(const std::vector<std::string>& texts, const std::vector<std::string>& vocab,
                                    int64_t max_len, bool lower, bool strip) {
  TORCH_CHECK(max_len >= 2, "text_encode: max_len >= 2");
  Vocab v;
  v.map.reserve(vocab.size() * 2);
  for (size_t i = 0; i < vocab.size(); ++i) v.map.emplace(vocab[i], (int64_t)i);
  auto get = [&](const char* t, int64_t d) { auto it = v.map.find(t); return it == v.map.end() ? d : it->second; };
  v.unk = get("[UNK]", 100);
  v.cls = get("[CLS]", 101);
  v.sep = get("[SEP]", 102);
  const int64_t N = (int64_t)texts.size();
  auto ids = at::zeros({N, max_len}, at::kLong);
  auto mask = at::zeros({N, max_len}, at::kLong);
  int64_t* ip = ids.data_ptr<int64_t>();
  int64_t* mp = mask.data_ptr<int64_t>();
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t n = 0; n < N; ++n) {
    std::vector<std::string> toks;
    basic_tokenize(strip ? strip_tags(texts[n]) : texts[n], lower, toks);
    std::vector<int64_t> wp;
    wp.reserve(toks.size() + 4);
    for (const auto& t : toks) {
      wordpiece(t, v, wp);
      if ((int64_t)wp.size() >= max_len) break;
    }
    const int64_t body = std::min<int64_t>((int64_t)wp.size(), max_len - 2);  // truncate (post)
    int64_t* row = ip + n * max_len;
    int64_t k = 0;
    row[k++] = v.cls;
    for (int64_t i = 0; i < body; ++i) row[k++] = wp[i];
    row[k++] = v.sep;
    for (int64_t i = 0; i < max_len; ++i) mp[n * max_len + i] = row[i] > 0 ? 1 : 0;  // padding 'post' = 0
  }
  return {ids, mask};
}

std::vector<std::string> text_basic_tokenize(const std::vector<std::string>& texts, bool lower, bool strip) {
  std::vector<std::string> out(texts.size());
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t n = 0; n < (int64_t)texts.size(); ++n) {
    std::vector<std::string> toks;
    basic_tokenize(strip ? strip_tags(texts[n]) : texts[n], lower, toks);
    std::string s;
    for (size_t i = 0; i < toks.size(); ++i) {
      if (i) s.push_back(' ');
      s += toks[i];
    }
    out[n] = std::move(s);
  }
  return out;
}

}  // namespace pcmp_rt

TORCH_LIBRARY_FRAGMENT(pcmp, m) {
  m.def("text_encode(str[] texts, str[] vocab, int max_len, bool lower, bool strip_tags) -> Tensor[]",
        &pcmp_rt::text_encode);
  m.def("text_basic_tokenize(str[] texts, bool lower, bool strip_tags) -> str[]", &pcmp_rt::text_basic_tokenize);
}
