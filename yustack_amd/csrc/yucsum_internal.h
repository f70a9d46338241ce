// yucsum_internal.h — library-internal entry points shared by the translation
// units of libyucsum.so. Not part of the C ABI (include/yucsum.h).
#ifndef YUCSUM_INTERNAL_H
#define YUCSUM_INTERNAL_H

#include <stdint.h>

// Enqueue on `stream` a one-thread kernel that stores `value` to `flag` (a
// device view of coherent pinned host memory) with system-scope fences, so a
// host thread polling the flag sees it only after everything enqueued before
// it on the stream has completed. Returns a YU_* status.
__attribute__((visibility("hidden"))) int yu_internal_signal(uint32_t *flag, uint32_t value,
                                                       void *stream);

#endif  // YUCSUM_INTERNAL_H
