/* ref_stbi.c — TEST INFRASTRUCTURE: the reference's own vendored JPEG/PNG loader
 * (external/stb_image.h v2.26, used by make_image / imread, texture.h:166-203), compiled in place
 * from /root/reference by `make -C oracle ref` into oracle/_ref/.  Tests use it to pin the texel
 * bytes of the product's image decoding; nothing in the product links it. */
#define STB_IMAGE_IMPLEMENTATION
#include "stb_image.h"

/* stbi_load(path, &w, &h, &channels_in_file, 0), as imread() calls it (texture.h:173). */
unsigned char* ref_stbi_load(const char* path, int* w, int* h, int* channels) {
  return stbi_load(path, w, h, channels, 0);
}
void ref_stbi_free(unsigned char* p) { stbi_image_free(p); }
