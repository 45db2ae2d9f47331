// song.cpp - native song ingestion behind include/pianosong.h (host C++17, init-time).
//
// MIDI bytes -> note sequence (pretty_midi pairing semantics, as note_seq uses them) ->
// fingering annotations -> trim_silence -> per-control-step song tables. Every ordering that
// can change a result (instrument order, stable sorts, tempo ties, last-write-wins of
// control changes) is the one of the reference's Python stack; see the header for the
// reference function each entry point restates.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "../../include/pianosong.h"

struct pss_seq {
  std::vector<pss_note> notes;
  std::vector<pss_cc> ccs;
  double total_time = 0.0;
};

namespace {

thread_local std::string g_err;
int fail(const std::string& s) {
  g_err = s;
  return -1;
}

constexpr int MIN_PITCH = 21, MAX_PITCH = 108, NKEYS = 88, SUSTAIN_CC = 64, MAX_CC = 127;
constexpr double MAX_VELOCITY = 127.0;

struct Reader {
  const uint8_t* d;
  size_t n, p = 0;
  bool ok = true;
  uint8_t u8() {
    if (p >= n) { ok = false; return 0; }
    return d[p++];
  }
  uint32_t be(int bytes) {
    uint32_t v = 0;
    for (int i = 0; i < bytes; i++) v = (v << 8) | u8();
    return v;
  }
  uint32_t varlen() {
    uint32_t v = 0;
    for (int i = 0; i < 4; i++) {
      const uint8_t b = u8();
      v = (v << 7) | (b & 0x7F);
      if (!(b & 0x80)) return v;
    }
    ok = false;
    return v;
  }
};

enum Kind { TEMPO, PROGRAM, NOTE_ON, NOTE_OFF, CC };
struct Event {
  uint64_t tick;
  Kind kind;
  int a, b, c;  // tempo: a = us/qn; program: ch, prog; note: ch, pitch, vel; cc: ch, num, val
};

int parse(const uint8_t* data, size_t len, pss_seq* seq) {
  Reader r{data, len};
  if (len < 14 || memcmp(data, "MThd", 4) != 0) return fail("not a Standard MIDI File");
  r.p = 4;
  const uint32_t hdr_len = r.be(4);
  r.be(2);  // format
  const int ntracks = (int)r.be(2);
  const int division = (int)r.be(2);
  if (division & 0x8000) return fail("SMPTE time division is not supported");
  if (division == 0) return fail("zero ticks per quarter note");
  size_t pos = 8 + (size_t)hdr_len;
  std::vector<std::vector<Event>> tracks;
  for (int t = 0; t < ntracks; t++) {
    if (pos + 8 > len || memcmp(data + pos, "MTrk", 4) != 0) return fail("bad track chunk");
    r.p = pos + 4;
    const size_t length = r.be(4);
    const size_t end = pos + 8 + length;
    if (end > len) return fail("truncated track chunk");
    Reader tr{data, end, pos + 8};
    uint64_t tick = 0;
    int status = 0;
    std::vector<Event> ev;
    while (tr.p < end) {
      tick += tr.varlen();
      const uint8_t b = tr.u8();
      if (!tr.ok) return fail("truncated event");
      if (b == 0xFF) {  // meta
        const uint8_t mtype = tr.u8();
        const uint32_t mlen = tr.varlen();
        if (!tr.ok || tr.p + mlen > end) return fail("truncated meta event");
        if (mtype == 0x51 && mlen >= 3)
          ev.push_back({tick, TEMPO, (data[tr.p] << 16) | (data[tr.p + 1] << 8) | data[tr.p + 2], 0, 0});
        tr.p += mlen;
        if (mtype == 0x2F) break;
        continue;
      }
      if (b == 0xF0 || b == 0xF7) {  // sysex
        const uint32_t slen = tr.varlen();
        tr.p += slen;
        continue;
      }
      int d1;
      if (b & 0x80) {
        status = b;
        d1 = tr.u8();
      } else {
        d1 = b;  // running status: b is the first data byte (status 0: two ignored data bytes)
      }
      const int kind = status & 0xF0, ch = status & 0x0F;
      if (kind == 0xC0 || kind == 0xD0) {
        if (kind == 0xC0) ev.push_back({tick, PROGRAM, ch, d1, 0});
        continue;
      }
      const int d2 = tr.u8();
      if (!tr.ok) return fail("truncated channel event");
      if (kind == 0x90) ev.push_back({tick, d2 > 0 ? NOTE_ON : NOTE_OFF, ch, d1, d2});
      else if (kind == 0x80) ev.push_back({tick, NOTE_OFF, ch, d1, d2});
      else if (kind == 0xB0) ev.push_back({tick, CC, ch, d1, d2});
    }
    if (!tr.ok) return fail("truncated track");
    tracks.push_back(std::move(ev));
    pos = end;
  }
  // tempo map from every track, sorted by (tick, value); the last change of a tick wins
  std::vector<std::pair<uint64_t, int>> tempos;
  for (auto& ev : tracks)
    for (auto& e : ev)
      if (e.kind == TEMPO) tempos.push_back({e.tick, e.a});
  std::sort(tempos.begin(), tempos.end());
  if (tempos.empty() || tempos[0].first != 0) tempos.insert(tempos.begin(), {0, 500000});
  std::vector<std::pair<uint64_t, int>> tmap;
  for (auto& tv : tempos) {
    if (!tmap.empty() && tmap.back().first == tv.first) tmap.back() = tv;
    else tmap.push_back(tv);
  }
  std::vector<double> seg(tmap.size(), 0.0);
  for (size_t i = 1; i < tmap.size(); i++) {
    const double dt_ticks = (double)(tmap[i].first - tmap[i - 1].first);
    seg[i] = seg[i - 1] + dt_ticks * tmap[i - 1].second / 1e6 / division;
  }
  auto tick_to_time = [&](uint64_t tick) {
    size_t i = tmap.size() - 1;
    while (tmap[i].first > tick) i--;
    return seg[i] + (double)(tick - tmap[i].first) * tmap[i].second / 1e6 / division;
  };
  // instruments keyed (track, channel, program), created on every note-off (first-seen order)
  std::map<std::tuple<int, int, int>, int> inst_index;
  std::vector<std::vector<pss_note>> instruments;
  for (size_t ti = 0; ti < tracks.size(); ti++) {
    int program[16] = {0};
    std::map<std::pair<int, int>, std::vector<std::pair<uint64_t, int>>> open;
    for (auto& e : tracks[ti]) {
      if (e.kind == PROGRAM) {
        program[e.a] = e.b;
      } else if (e.kind == NOTE_ON) {
        open[{e.a, e.b}].push_back({e.tick, e.c});
      } else if (e.kind == NOTE_OFF) {
        auto it = open.find({e.a, e.b});
        if (it == open.end()) continue;
        std::vector<std::pair<uint64_t, int>> close, keep;
        for (auto& sv : it->second) (sv.first != e.tick ? close : keep).push_back(sv);
        const auto key = std::make_tuple((int)ti, e.a, program[e.a]);
        auto ii = inst_index.find(key);
        if (ii == inst_index.end()) {
          ii = inst_index.emplace(key, (int)instruments.size()).first;
          instruments.emplace_back();
        }
        for (auto& sv : close)
          instruments[ii->second].push_back({e.b, tick_to_time(sv.first), tick_to_time(e.tick), sv.second, 0});
        if (!close.empty() && !keep.empty()) it->second = keep;
        else if (!close.empty()) open.erase(it);
      } else if (e.kind == CC) {
        seq->ccs.push_back({tick_to_time(e.tick), e.b, e.c});
      }
    }
  }
  for (auto& inst : instruments) seq->notes.insert(seq->notes.end(), inst.begin(), inst.end());
  seq->total_time = 0.0;
  for (auto& nt : seq->notes) seq->total_time = std::max(seq->total_time, nt.end_time);
  return 0;
}

// "C#4" -> 61 (add_fingering_to_midi.py:7-24: regex ([A-G][#b]?)(\d+) at the start)
bool pitch_number(const std::string& s, int* out) {
  if (s.empty() || s[0] < 'A' || s[0] > 'G') return false;
  static const int base[7] = {9, 11, 0, 2, 4, 5, 7};  // A B C D E F G
  int v = base[s[0] - 'A'];
  size_t i = 1;
  if (i < s.size() && (s[i] == '#' || s[i] == 'b')) {
    // the reference's table only has C# Db D# Eb F# Gb G# Ab A# Bb (E#/Fb/B#/Cb raise KeyError)
    const char n = s[0], acc = s[i];
    const bool ok = acc == '#' ? (n == 'C' || n == 'D' || n == 'F' || n == 'G' || n == 'A')
                               : (n == 'D' || n == 'E' || n == 'G' || n == 'A' || n == 'B');
    if (!ok) return false;
    v += acc == '#' ? 1 : -1;
    i++;
  }
  size_t j = i;
  while (j < s.size() && s[j] >= '0' && s[j] <= '9') j++;
  if (j == i) return false;
  *out = v + (atoi(s.substr(i, j - i).c_str()) + 1) * 12;
  return true;
}

std::string strip(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && isspace((unsigned char)s[a])) a++;
  while (b > a && isspace((unsigned char)s[b - 1])) b--;
  return s.substr(a, b - a);
}

bool to_double(const std::string& s, double* out) {
  const std::string t = strip(s);
  if (t.empty()) return false;
  char* e = nullptr;
  *out = strtod(t.c_str(), &e);
  return e && *e == '\0';
}

bool to_int(const std::string& s, long* out) {
  const std::string t = strip(s);
  if (t.empty()) return false;
  char* e = nullptr;
  *out = strtol(t.c_str(), &e, 10);
  return e && *e == '\0';
}

}  // namespace

extern "C" {

const char* pss_last_error(void) { return g_err.c_str(); }
int pss_version(void) { return 1; }

int pss_parse_midi(const uint8_t* data, size_t len, pss_seq** out) {
  if (!data || !out) return fail("pss_parse_midi: null argument");
  auto* s = new pss_seq();
  const int rc = parse(data, len, s);
  if (rc) {
    delete s;
    return rc;
  }
  *out = s;
  return 0;
}

int pss_from_notes(const pss_note* notes, int n_notes, const pss_cc* ccs, int n_cc, double total_time, pss_seq** out) {
  if (!out || n_notes < 0 || n_cc < 0 || (n_notes && !notes) || (n_cc && !ccs)) return fail("pss_from_notes: bad argument");
  auto* s = new pss_seq();
  s->notes.assign(notes, notes + n_notes);
  s->ccs.assign(ccs, ccs + n_cc);
  s->total_time = total_time;
  *out = s;
  return 0;
}

void pss_free(pss_seq* seq) { delete seq; }

int pss_info(const pss_seq* s, int* n_notes, int* n_cc, double* total_time, int* has_fingering) {
  if (!s) return fail("pss_info: null sequence");
  if (n_notes) *n_notes = (int)s->notes.size();
  if (n_cc) *n_cc = (int)s->ccs.size();
  if (total_time) *total_time = s->total_time;
  if (has_fingering) {  // MidiFile.has_fingering (midi_file.py:252-261)
    std::vector<int> parts;
    for (auto& n : s->notes) parts.push_back(n.part);
    std::sort(parts.begin(), parts.end());
    parts.erase(std::unique(parts.begin(), parts.end()), parts.end());
    bool nonzero = false;
    for (int p : parts) nonzero |= p != 0;
    *has_fingering = parts.size() > 1 && nonzero;
  }
  return 0;
}

int pss_get(const pss_seq* s, pss_note* notes, pss_cc* ccs) {
  if (!s) return fail("pss_get: null sequence");
  if (notes) std::copy(s->notes.begin(), s->notes.end(), notes);
  if (ccs) std::copy(s->ccs.begin(), s->ccs.end(), ccs);
  return 0;
}

// each note takes the finger of the first annotation line whose start and end are within
// 10 ms and whose pitch is equal (add_fingering_to_midi.py:55-80)
int pss_add_fingering(pss_seq* s, const char* text) {
  if (!s || !text) return fail("pss_add_fingering: null argument");
  struct Ann { double start, end; int pitch; long finger; };
  std::vector<Ann> ann;
  std::string all(text);
  size_t p = 0;
  while (p <= all.size()) {
    size_t q = all.find('\n', p);
    if (q == std::string::npos) q = all.size();
    std::string line = all.substr(p, q - p);
    if (!line.empty() && line.back() == '\r') line.pop_back();  // str.splitlines
    p = q + 1;
    if (line.rfind("//", 0) == 0 || strip(line).empty()) continue;
    const std::string st = strip(line);
    std::vector<std::string> parts;
    size_t a = 0;
    while (true) {
      const size_t b = st.find('\t', a);
      parts.push_back(st.substr(a, b == std::string::npos ? std::string::npos : b - a));
      if (b == std::string::npos) break;
      a = b + 1;
    }
    if (parts.size() != 8) continue;
    long f;
    double t0, t1;
    int pitch;
    if (!to_int(parts[7], &f)) return fail("annotation: bad finger '" + parts[7] + "'");
    if (f < 0 || f > 9) continue;
    if (!to_double(parts[1], &t0) || !to_double(parts[2], &t1)) return fail("annotation: bad time in '" + st + "'");
    if (!pitch_number(parts[3], &pitch)) return fail("Invalid pitch format: " + parts[3]);
    ann.push_back({t0, t1, pitch, f});
  }
  for (auto& n : s->notes)
    for (auto& a : ann)
      if (fabs(n.start_time - a.start) < 0.01 && fabs(n.end_time - a.end) < 0.01 && n.pitch == a.pitch) {
        n.part = (int)a.finger;
        break;
      }
  return 0;
}

// extract_subsequence(seq, notes[0].start, notes[-1].end) (midi_file.py:231-237)
int pss_trim_silence(pss_seq* s) {
  if (!s) return fail("pss_trim_silence: null sequence");
  pss_seq out;
  if (s->notes.empty()) {
    *s = out;
    return 0;
  }
  const double start = s->notes.front().start_time, end = s->notes.back().end_time;
  std::vector<pss_note> sorted = s->notes;
  std::stable_sort(sorted.begin(), sorted.end(),
                   [](const pss_note& a, const pss_note& b) { return a.start_time < b.start_time; });
  for (auto& n : sorted) {
    if (n.start_time < start || n.start_time >= end) continue;
    const double e = std::min(n.end_time, end) - start;
    out.notes.push_back({n.pitch, n.start_time - start, e, n.velocity, n.part});
    out.total_time = std::max(out.total_time, e);
  }
  std::vector<pss_cc> cs = s->ccs;
  std::stable_sort(cs.begin(), cs.end(), [](const pss_cc& a, const pss_cc& b) { return a.time < b.time; });
  int pedal = -1;
  for (auto& c : cs) {
    if (c.time < start) {
      if (c.control_number == SUSTAIN_CC) pedal = c.control_value;
      continue;
    }
    if (c.time >= end) continue;
    out.ccs.push_back({c.time - start, c.control_number, c.control_value});
  }
  if (pedal >= 64) out.ccs.insert(out.ccs.begin(), {0.0, SUSTAIN_CC, pedal});
  *s = std::move(out);
  return 0;
}

int pss_song_tables(const pss_seq* s, double dt, double initial_buffer_time, int max_T, int max_notes, float* goal,
                    int32_t* count, int32_t* keys, int32_t* fingers, int* T_out) {
  if (!s || !T_out) return fail("pss_song_tables: null argument");
  if (!(dt > 0)) return fail("pss_song_tables: dt must be positive");
  if (initial_buffer_time < 0) return fail("initial_buffer_time must be non-negative.");
  const double fps = 1.0 / dt;
  const long nf = (long)(s->total_time * fps + 1);
  if (nf < 1 || nf > (1L << 24)) return fail("pss_song_tables: song length out of range");
  const size_t F = (size_t)nf;
  std::vector<float> vel(F * 128, 0.f), onset(F * 128, 0.f), finger(F * 128, -1.f);
  std::vector<int> cc(F * 128, 0);
  auto frames = [&](double a, double b, long* sf, long* ef) {
    *sf = (long)(a * fps);
    const long e = (long)ceil(b * fps);
    *ef = std::max(*sf + 1, e);
  };
  std::vector<pss_note> sorted = s->notes;
  std::stable_sort(sorted.begin(), sorted.end(),
                   [](const pss_note& a, const pss_note& b) { return a.start_time < b.start_time; });
  for (auto& n : sorted) {
    if (n.pitch < 0 || n.pitch > 127) continue;
    long sf, ef;
    frames(n.start_time, n.end_time, &sf, &ef);
    if (sf >= 0 && sf < nf) onset[(size_t)sf * 128 + n.pitch] = 1.f;
    const float v = (float)(n.velocity / MAX_VELOCITY);
    for (long t = std::max(sf, 0L); t < std::min(ef, nf); t++) {
      vel[(size_t)t * 128 + n.pitch] = v;
      finger[(size_t)t * 128 + n.pitch] = (float)n.part;
    }
  }
  for (auto& c : s->ccs) {
    long f, e;
    frames(c.time, 0.0, &f, &e);
    if (f < nf && f >= 0 && c.control_number >= 0 && c.control_number < 128)
      cc[(size_t)f * 128 + c.control_number] = c.control_value + 1;
  }
  const long nbuf = (long)nearbyint(initial_buffer_time / dt);  // Python round(): half to even
  const long T = nbuf + nf;
  *T_out = (int)T;
  if (!goal) return 0;
  if (T > max_T) return fail("pss_song_tables: max_T too small");
  if (!count || !keys || !fingers || max_notes <= 0) return fail("pss_song_tables: null table");
  memset(goal, 0, sizeof(float) * (size_t)T * (NKEYS + 1));
  for (long t = 0; t < T; t++) {
    count[t] = 0;
    for (int i = 0; i < max_notes; i++) keys[t * max_notes + i] = fingers[t * max_notes + i] = -1;
  }
  int prev = 0;
  for (long f = 0; f < nf; f++) {
    const long t = f + nbuf;
    int c = 0;
    for (int p = 0; p < 128; p++) {
      const float v = vel[(size_t)f * 128 + p];
      if (v == 0.f) continue;
      // a re-strike in its onset frame leaves a gap (piano_roll.py onset handling)
      if (f > 0 && vel[(size_t)(f - 1) * 128 + p] != 0.f && v * onset[(size_t)f * 128 + p] != 0.f) continue;
      if (p < MIN_PITCH || p > MAX_PITCH) return fail("pitch " + std::to_string(p) + " outside the piano range");
      if (c >= max_notes)
        return fail("step " + std::to_string(t) + " has more than " + std::to_string(max_notes) + " notes");
      keys[t * max_notes + c] = p - MIN_PITCH;
      fingers[t * max_notes + c] = (int)finger[(size_t)f * 128 + p];
      goal[(size_t)t * (NKEYS + 1) + (p - MIN_PITCH)] = 1.f;
      c++;
    }
    count[t] = c;
    const int ev = cc[(size_t)f * 128 + SUSTAIN_CC];
    int sus;
    if (1 <= ev && ev <= SUSTAIN_CC) sus = 0;
    else if (SUSTAIN_CC + 1 <= ev && ev <= MAX_CC + 1) sus = 1;
    else sus = prev;
    prev = sus;
    goal[(size_t)t * (NKEYS + 1) + NKEYS] = (float)sus;
  }
  return 0;
}

}  // extern "C"
