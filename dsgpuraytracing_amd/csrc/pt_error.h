// pt_error.h — shared error reporting of libptgpu.so: every C-ABI failure sets
// a thread-local message (pt_last_error) and returns a negative PT_E_* code.
#pragma once
#include <string>

int pt_fail(int code, const std::string& msg);
