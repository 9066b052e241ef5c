// Host sanitizer harness for the native text pipeline core (csrc/runtime/text_core.h), built by
// tests/test_native_sanitizers_cpu.py with -fsanitize=address,undefined (sanitizers
// on host-side extension code; GPU sanitizers are not available on this pool).  Exercises the
// edge cases of the tokenizer / WordPiece / row encoder and checks exact outputs; any sanitizer
// report or failed check exits non-zero.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "runtime/text_core.h"

using namespace pcmp_rt;

static int fails = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "CHECK failed line %d: %s\n", __LINE__, #c); \
      ++fails;                                                     \
    }                                                              \
  } while (0)

int main() {
  Vocab v;
  const char* words[] = {"[PAD]", "the", "movie", "was", "great", "##s", "great", "!", ",", "un", "##believ", "##able"};
  for (int i = 0; i < (int)(sizeof(words) / sizeof(words[0])); ++i) v.map.emplace(words[i], 1000 + i);
  v.unk = 100; v.cls = 101; v.sep = 102;

  // tag stripping: closed tags -> one space, unterminated '<' kept, empty '<>' kept
  CHECK(strip_tags("a<br />b") == "a b");
  CHECK(strip_tags("x < y") == "x < y");
  CHECK(strip_tags("<>") == "<>");
  CHECK(strip_tags("") == "");
  CHECK(strip_tags("<<a>") == " ");          // regex <[^>]+> matches "<<a>" whole

  std::vector<std::string> t;
  basic_tokenize("The Movie,was GREAT!", true, t);
  CHECK(t.size() == 6 && t[0] == "the" && t[2] == "," && t[5] == "!");
  t.clear();
  basic_tokenize(std::string("caf\xc3\xa9 \x00x", 8), true, t);   // accent stripped (lower), NUL dropped
  CHECK(t.size() == 2 && t[0] == "cafe" && t[1] == "x");
  t.clear();
  basic_tokenize(std::string("caf\xc3\xa9", 5), false, t);   // no lower-casing: accents kept
  CHECK(t.size() == 1 && t[0] == "caf\xc3\xa9");
  t.clear();
  basic_tokenize("\xe4\xb8\xad\xe5\x9b\xbd" "ab\xe2\x80\x94" "c \xc3\x80", true, t);   // CJK isolated, em dash is P*
  CHECK(t.size() == 6 && t[2] == "ab" && t[3] == "\xe2\x80\x94" && t[4] == "c" && t[5] == "a");
  t.clear();
  basic_tokenize(std::string("a\xe2\x80\x8b" "b\xc3", 6), true, t);   // zero-width space (Cf) dropped, truncated UTF-8 dropped
  CHECK(t.size() == 1 && t[0] == "ab");

  std::vector<int64_t> wp;
  wordpiece("unbelievable", v, wp);
  CHECK(wp.size() == 3 && wp[0] == 1009 && wp[1] == 1010 && wp[2] == 1011);
  wp.clear();
  wordpiece("xyz", v, wp);
  CHECK(wp.size() == 1 && wp[0] == v.unk);
  wp.clear();
  wordpiece(std::string(101, 'a'), v, wp);   // > 100 chars -> [UNK]
  CHECK(wp.size() == 1 && wp[0] == v.unk);

  // row encoder: truncation at every max_len from the minimum up, padding and mask
  const std::string review = "<b>The movie</b> was great, great great!" + std::string(300, ' ') + std::string(5000, 'z');
  for (int64_t L = 2; L <= 20; ++L) {
    std::vector<int64_t> row(L, -7), mask(L, -7);
    encode_row(review, v, L, true, true, row.data(), mask.data());
    CHECK(row[0] == v.cls);
    int64_t k = 1;
    while (k < L && row[k] != v.sep) ++k;
    CHECK(k < L);
    for (int64_t i = k + 1; i < L; ++i) CHECK(row[i] == 0);
    for (int64_t i = 0; i < L; ++i) CHECK(mask[i] == (row[i] > 0 ? 1 : 0));
  }
  std::vector<int64_t> row(8), mask(8);
  encode_row("", v, 8, true, true, row.data(), mask.data());
  CHECK(row[0] == v.cls && row[1] == v.sep && row[2] == 0 && mask[1] == 1 && mask[2] == 0);

  if (fails) {
    std::fprintf(stderr, "%d check(s) failed\n", fails);
    return 1;
  }
  std::printf("text_core_check: ok\n");
  return 0;
}
