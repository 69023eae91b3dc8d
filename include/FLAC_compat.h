/*
 * FLAC_compat.h -- libFLAC 1.2.1 stream-decoder ABI types, as BirdNest.Audio binds them.
 *
 * These are the enums, callback signatures and struct layouts that the reference's
 * P/Invoke layer marshals (Library/LibFLACSharp/LibFLACSharp.cs).  Both the MI355X
 * decoder (libbnflac.so, include/bnflac.h) and the CPU oracle (oracle/) use them, so
 * the byte offsets the C# reads are pinned in one place and checked by
 * tests/test_abi.py against the C# FieldOffsets:
 *
 *   FLAC__FrameHeader  <-> LibFLAC.FrameHeader     LibFLACSharp.cs:224-234
 *       blocksize@0 sample_rate@4 channels@8 channel_assignment@12
 *       bits_per_sample@16 number_type@20 number@24 crc@32
 *   FLAC__StreamMetadata <-> LibFLAC.FLACMetaData  LibFLACSharp.cs:282-293
 *       type@0 is_last@4 length@8 data@16 (C# Data[] starts at 12, so the C#
 *       FLACStreamInfo FieldOffset(4) lands on min_blocksize@16)
 *   FLAC__StreamMetadata_StreamInfo <-> LibFLAC.FLACStreamInfo LibFLACSharp.cs:295-319
 *       sample_rate@32 channels@36 bits_per_sample@40 (pad@44 == C# "TotalSamplesHi")
 *       total_samples@48 (low word == C# "TotalSamplesLo") md5sum@56
 *
 * Enum values follow LibFLACSharp.cs:24-36 (StreamDecoderState), :89-173 (status
 * codes) and :262-268 (DecodeError).  The layouts are identical on x86 and x86-64
 * (no pointer precedes a marshalled field).
 */
#ifndef BNFLAC_FLAC_COMPAT_H
#define BNFLAC_FLAC_COMPAT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int FLAC__bool;
typedef uint8_t FLAC__byte;
typedef uint8_t FLAC__uint8;
typedef uint16_t FLAC__uint16;
typedef int32_t FLAC__int32;
typedef uint32_t FLAC__uint32;
typedef int64_t FLAC__int64;
typedef uint64_t FLAC__uint64;

#define FLAC__MAX_CHANNELS 8u
#define FLAC__MAX_FIXED_ORDER 4u
#define FLAC__MAX_LPC_ORDER 32u

/* LibFLACSharp.cs:24-36 */
typedef enum {
    FLAC__STREAM_DECODER_SEARCH_FOR_METADATA = 0,
    FLAC__STREAM_DECODER_READ_METADATA,
    FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC,
    FLAC__STREAM_DECODER_READ_FRAME,
    FLAC__STREAM_DECODER_END_OF_STREAM,
    FLAC__STREAM_DECODER_OGG_ERROR,
    FLAC__STREAM_DECODER_SEEK_ERROR,
    FLAC__STREAM_DECODER_ABORTED,
    FLAC__STREAM_DECODER_MEMORY_ALLOCATION_ERROR,
    FLAC__STREAM_DECODER_UNINITIALIZED
} FLAC__StreamDecoderState;

typedef enum {
    FLAC__STREAM_DECODER_INIT_STATUS_OK = 0,
    FLAC__STREAM_DECODER_INIT_STATUS_UNSUPPORTED_CONTAINER,
    FLAC__STREAM_DECODER_INIT_STATUS_INVALID_CALLBACKS,
    FLAC__STREAM_DECODER_INIT_STATUS_MEMORY_ALLOCATION_ERROR,
    FLAC__STREAM_DECODER_INIT_STATUS_ERROR_OPENING_FILE,
    FLAC__STREAM_DECODER_INIT_STATUS_ALREADY_INITIALIZED
} FLAC__StreamDecoderInitStatus;

/* LibFLACSharp.cs:89-110 */
typedef enum {
    FLAC__STREAM_DECODER_READ_STATUS_CONTINUE = 0,
    FLAC__STREAM_DECODER_READ_STATUS_END_OF_STREAM,
    FLAC__STREAM_DECODER_READ_STATUS_ABORT
} FLAC__StreamDecoderReadStatus;

/* LibFLACSharp.cs:113-127 */
typedef enum {
    FLAC__STREAM_DECODER_SEEK_STATUS_OK = 0,
    FLAC__STREAM_DECODER_SEEK_STATUS_ERROR,
    FLAC__STREAM_DECODER_SEEK_STATUS_UNSUPPORTED
} FLAC__StreamDecoderSeekStatus;

/* LibFLACSharp.cs:130-144 */
typedef enum {
    FLAC__STREAM_DECODER_TELL_STATUS_OK = 0,
    FLAC__STREAM_DECODER_TELL_STATUS_ERROR,
    FLAC__STREAM_DECODER_TELL_STATUS_UNSUPPORTED
} FLAC__StreamDecoderTellStatus;

/* LibFLACSharp.cs:147-161 */
typedef enum {
    FLAC__STREAM_DECODER_LENGTH_STATUS_OK = 0,
    FLAC__STREAM_DECODER_LENGTH_STATUS_ERROR,
    FLAC__STREAM_DECODER_LENGTH_STATUS_UNSUPPORTED
} FLAC__StreamDecoderLengthStatus;

/* LibFLACSharp.cs:163-173 */
typedef enum {
    FLAC__STREAM_DECODER_WRITE_STATUS_CONTINUE = 0,
    FLAC__STREAM_DECODER_WRITE_STATUS_ABORT
} FLAC__StreamDecoderWriteStatus;

/* LibFLACSharp.cs:262-268 */
typedef enum {
    FLAC__STREAM_DECODER_ERROR_STATUS_LOST_SYNC = 0,
    FLAC__STREAM_DECODER_ERROR_STATUS_BAD_HEADER,
    FLAC__STREAM_DECODER_ERROR_STATUS_FRAME_CRC_MISMATCH,
    FLAC__STREAM_DECODER_ERROR_STATUS_UNPARSEABLE_STREAM
} FLAC__StreamDecoderErrorStatus;

typedef enum {
    FLAC__CHANNEL_ASSIGNMENT_INDEPENDENT = 0,
    FLAC__CHANNEL_ASSIGNMENT_LEFT_SIDE = 1,
    FLAC__CHANNEL_ASSIGNMENT_RIGHT_SIDE = 2,
    FLAC__CHANNEL_ASSIGNMENT_MID_SIDE = 3
} FLAC__ChannelAssignment;

typedef enum {
    FLAC__FRAME_NUMBER_TYPE_FRAME_NUMBER = 0,
    FLAC__FRAME_NUMBER_TYPE_SAMPLE_NUMBER
} FLAC__FrameNumberType;

typedef enum {
    FLAC__SUBFRAME_TYPE_CONSTANT = 0,
    FLAC__SUBFRAME_TYPE_VERBATIM = 1,
    FLAC__SUBFRAME_TYPE_FIXED = 2,
    FLAC__SUBFRAME_TYPE_LPC = 3
} FLAC__SubframeType;

typedef enum {
    FLAC__ENTROPY_CODING_METHOD_PARTITIONED_RICE = 0,
    FLAC__ENTROPY_CODING_METHOD_PARTITIONED_RICE2 = 1
} FLAC__EntropyCodingMethodType;

typedef enum {
    FLAC__METADATA_TYPE_STREAMINFO = 0,
    FLAC__METADATA_TYPE_PADDING = 1,
    FLAC__METADATA_TYPE_APPLICATION = 2,
    FLAC__METADATA_TYPE_SEEKTABLE = 3,
    FLAC__METADATA_TYPE_VORBIS_COMMENT = 4,
    FLAC__METADATA_TYPE_CUESHEET = 5,
    FLAC__METADATA_TYPE_PICTURE = 6,
    FLAC__METADATA_TYPE_UNDEFINED = 7
} FLAC__MetadataType;

/* LibFLACSharp.cs:224-234 */
typedef struct {
    unsigned blocksize;
    unsigned sample_rate;
    unsigned channels;
    FLAC__ChannelAssignment channel_assignment;
    unsigned bits_per_sample;
    FLAC__FrameNumberType number_type;
    union {
        FLAC__uint32 frame_number;
        FLAC__uint64 sample_number;
    } number;
    FLAC__uint8 crc;
} FLAC__FrameHeader;

typedef struct {
    unsigned *parameters;
    unsigned *raw_bits;
    unsigned capacity_by_order;
} FLAC__EntropyCodingMethod_PartitionedRiceContents;

typedef struct {
    unsigned order;
    const FLAC__EntropyCodingMethod_PartitionedRiceContents *contents;
} FLAC__EntropyCodingMethod_PartitionedRice;

typedef struct {
    FLAC__EntropyCodingMethodType type;
    union {
        FLAC__EntropyCodingMethod_PartitionedRice partitioned_rice;
    } data;
} FLAC__EntropyCodingMethod;

typedef struct { FLAC__int32 value; } FLAC__Subframe_Constant;
typedef struct { const FLAC__int32 *data; } FLAC__Subframe_Verbatim;

typedef struct {
    FLAC__EntropyCodingMethod entropy_coding_method;
    unsigned order;
    FLAC__int32 warmup[FLAC__MAX_FIXED_ORDER];
    const FLAC__int32 *residual;
} FLAC__Subframe_Fixed;

typedef struct {
    FLAC__EntropyCodingMethod entropy_coding_method;
    unsigned order;
    unsigned qlp_coeff_precision;
    int quantization_level;
    FLAC__int32 qlp_coeff[FLAC__MAX_LPC_ORDER];
    FLAC__int32 warmup[FLAC__MAX_LPC_ORDER];
    const FLAC__int32 *residual;
} FLAC__Subframe_LPC;

typedef struct {
    FLAC__SubframeType type;
    union {
        FLAC__Subframe_Constant constant;
        FLAC__Subframe_Fixed fixed;
        FLAC__Subframe_LPC lpc;
        FLAC__Subframe_Verbatim verbatim;
    } data;
    unsigned wasted_bits;
} FLAC__Subframe;

typedef struct { FLAC__uint16 crc; } FLAC__FrameFooter;

typedef struct {
    FLAC__FrameHeader header;
    FLAC__Subframe subframes[FLAC__MAX_CHANNELS];
    FLAC__FrameFooter footer;
} FLAC__Frame;

/* LibFLACSharp.cs:295-319 */
typedef struct {
    unsigned min_blocksize, max_blocksize;
    unsigned min_framesize, max_framesize;
    unsigned sample_rate;
    unsigned channels;
    unsigned bits_per_sample;
    FLAC__uint64 total_samples;
    FLAC__byte md5sum[16];
} FLAC__StreamMetadata_StreamInfo;

/* LibFLACSharp.cs:282-293.  The C# marshals 12 + 100 bytes from this pointer, so the
 * union is padded the way libFLAC's larger members (cue sheet, picture) pad it. */
typedef struct {
    FLAC__MetadataType type;
    FLAC__bool is_last;
    unsigned length;
    union {
        FLAC__StreamMetadata_StreamInfo stream_info;
        FLAC__byte _reserved[160];
    } data;
} FLAC__StreamMetadata;

struct FLAC__StreamDecoder;
typedef struct FLAC__StreamDecoder FLAC__StreamDecoder;

/* LibFLACSharp.cs:187-212 */
typedef FLAC__StreamDecoderReadStatus (*FLAC__StreamDecoderReadCallback)(
    const FLAC__StreamDecoder *decoder, FLAC__byte buffer[], size_t *bytes, void *client_data);
typedef FLAC__StreamDecoderSeekStatus (*FLAC__StreamDecoderSeekCallback)(
    const FLAC__StreamDecoder *decoder, FLAC__uint64 absolute_byte_offset, void *client_data);
typedef FLAC__StreamDecoderTellStatus (*FLAC__StreamDecoderTellCallback)(
    const FLAC__StreamDecoder *decoder, FLAC__uint64 *absolute_byte_offset, void *client_data);
typedef FLAC__StreamDecoderLengthStatus (*FLAC__StreamDecoderLengthCallback)(
    const FLAC__StreamDecoder *decoder, FLAC__uint64 *stream_length, void *client_data);
typedef FLAC__bool (*FLAC__StreamDecoderEofCallback)(const FLAC__StreamDecoder *decoder,
                                                      void *client_data);
typedef FLAC__StreamDecoderWriteStatus (*FLAC__StreamDecoderWriteCallback)(
    const FLAC__StreamDecoder *decoder, const FLAC__Frame *frame,
    const FLAC__int32 *const buffer[], void *client_data);
typedef void (*FLAC__StreamDecoderMetadataCallback)(const FLAC__StreamDecoder *decoder,
                                                     const FLAC__StreamMetadata *metadata,
                                                     void *client_data);
typedef void (*FLAC__StreamDecoderErrorCallback)(const FLAC__StreamDecoder *decoder,
                                                  FLAC__StreamDecoderErrorStatus status,
                                                  void *client_data);

#ifdef __cplusplus
}
#endif

#endif /* BNFLAC_FLAC_COMPAT_H */
