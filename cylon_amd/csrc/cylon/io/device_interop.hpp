// Arrow C Device Data Interface for device tables (zero-copy hand-off to and from
// other Arrow-device consumers: ARROW_DEVICE_ROCM arrays whose buffers stay in HBM).
//
// Reference: the reference builds tables zero-copy from raw (address, size) buffers
// (arrow/arrow_builder.cpp:31-161; Java ArrowTable.cpp:185-270) but has no device
// memory.  Export here is a struct array ("+s") of the columns: fixed-width values,
// int64 string offsets ("U"/"Z"), bytes and list child values are the column's own
// HBM buffers; only what the layouts differ in is produced on the device (Arrow
// validity bitmaps from the byte masks by one ballot per 64 rows, bit-packed
// booleans, element offsets of list columns).  `sync_event` is a hipEvent_t recorded
// after those kernels.  Import wraps the producer's buffers as tensors that keep the
// producer's array alive (released when the last column buffer dies).
#pragma once
#include <arrow/c/abi.h>

#include "../table.hpp"

namespace cylon {
namespace io {

// Fills *schema / *array (caller-owned structs; released through their callbacks).
void ExportDeviceTable(const TablePtr &t, ArrowSchema *schema, ArrowDeviceArray *array);
// Moves *schema / *array into a table on `ctx` (the structs are released / marked released).
TablePtr ImportDeviceTable(const std::shared_ptr<CylonContext> &ctx, ArrowSchema *schema, ArrowDeviceArray *array);

}  // namespace io
}  // namespace cylon
