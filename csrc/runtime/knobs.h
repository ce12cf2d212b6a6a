// Tuning and diagnostic knobs of the native layer, in one documented registry.
//
// SURVEY.md §5 "Config": every setting has one home.  Python's `Config.native_knobs`
// (oap_mllib_amd/config.py) holds them for a process and `init_world` installs them here
// (`set_knob`); a knob not set there falls back to the process environment, which this file
// alone reads (tests switch knobs with monkeypatch.setenv between calls, so a value is looked up
// at each use, never cached).  Every knob the native code consults must be listed in
// `knob_table()` with its default and meaning: an unknown name is a programming error
// (ConfigError), so the table is the complete list (docs/ARCHITECTURE.md "Knobs").
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace oap {

struct KnobInfo {
  const char* name;
  const char* def;  // default value ("" = unset)
  const char* doc;
};

const std::vector<KnobInfo>& knob_table();

// The knob's value: the installed override, else the environment, else its default.
std::string knob_str(const char* name);
// ... as an integer / a floating-point value (an empty or non-numeric value reads as the default)
int64_t knob_int(const char* name);
double knob_float(const char* name);
// Set to a non-empty value other than "0" (flags whose default is off).
bool knob_on(const char* name);

// Installs (value non-empty) or removes (empty) an override; unknown names throw.
void set_knob(const std::string& name, const std::string& value);
void clear_knobs();

}  // namespace oap
