// C ABI version of the native libraries (checked by ops/_native.py at load time). Bump it whenever a
// launcher's argument list changes, together with ABI_VERSION in ops/_native.py.
#pragma once
#define H2O_ABI_VERSION 14
