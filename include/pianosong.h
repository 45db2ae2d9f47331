/*
 * pianosong.h - C-ABI of the native song ingestion: MIDI
 * file -> note sequence -> the per-control-step song tables ps_create consumes.
 *
 * The reference does this in Python on top of note_seq / pretty_midi (neither is
 * installable here); each entry point restates one reference function, with the
 * semantics of the library call underneath it:
 *
 *   pss_parse_midi      <- MidiFile.from_file / note_seq.midi_file_to_note_sequence
 *                          (robopianist/music/midi_file.py:179; pretty_midi's note pairing:
 *                          an off closes every open (channel, pitch) note started at an
 *                          earlier tick; instruments keyed (track, channel, program) in
 *                          first-seen order; merged tempo map, default 120 qpm).
 *   pss_add_fingering   <- add_fingering_from_annotation_file
 *                          (data_processing/add_fingering_to_midi.py:26-83).
 *   pss_trim_silence    <- MidiFile.trim_silence (midi_file.py:231-237) with
 *                          note_seq.sequences_lib.extract_subsequence semantics.
 *   pss_song_tables     <- NoteTrajectory.seq_to_trajectory (midi_file.py:315-362) over
 *                          sequence_to_pianoroll (piano_roll.py:59-204, onset_window 0),
 *                          add_initial_buffer_time (midi_file.py:388-401), and the goal /
 *                          finger tables of piano_with_shadow_hands.py:371-412.
 *
 * Host memory only (init-time work). 0 = OK, < 0 = error, message in pss_last_error()
 * (thread-local), e.g. a truncated file, an SMPTE division, a pitch outside the piano,
 * an annotation line with a malformed pitch.
 */
#ifndef PIANOSONG_H
#define PIANOSONG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int32_t pitch;
  double start_time, end_time;
  int32_t velocity;
  int32_t part; /* fingering: 0-4 right hand, 5-9 left hand (note_seq Note.part) */
} pss_note;

typedef struct {
  double time;
  int32_t control_number, control_value;
} pss_cc;

typedef struct pss_seq pss_seq; /* owns a note sequence */

const char* pss_last_error(void);
int pss_version(void);

int pss_parse_midi(const uint8_t* data, size_t len, pss_seq** out);
int pss_from_notes(const pss_note* notes, int n_notes, const pss_cc* ccs, int n_cc, double total_time, pss_seq** out);
void pss_free(pss_seq* seq);

/* sizes, then copy-out (either array may be NULL) */
int pss_info(const pss_seq* seq, int* n_notes, int* n_cc, double* total_time, int* has_fingering);
int pss_get(const pss_seq* seq, pss_note* notes, pss_cc* ccs);

int pss_add_fingering(pss_seq* seq, const char* annotation_text);
int pss_trim_silence(pss_seq* seq);

/* Tables of T control steps: goal [T][89] (keys active at t, then the sustain target),
 * count [T], keys / fingers [T][max_notes] (pitch order, -1 padded). Call with goal == NULL
 * to get T only; otherwise T must be <= max_T. */
int pss_song_tables(const pss_seq* seq, double dt, double initial_buffer_time, int max_T, int max_notes,
                    float* goal, int32_t* count, int32_t* keys, int32_t* fingers, int* T);

#ifdef __cplusplus
}
#endif
#endif
