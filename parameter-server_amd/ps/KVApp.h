// ps/KVApp.h — the include name the reference harnesses use (tests/src/LRServer.h:5).
#pragma once
#include "ps/kv_app.h"
