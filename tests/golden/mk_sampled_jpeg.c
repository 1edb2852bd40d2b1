/* Test infrastructure (tests/golden/gen_recovery_golden.py): writes a baseline
 * JPEG with luma sampling factors (h, v) and 1x1 chroma through IJG libjpeg
 * 9's encoder (/opt/conda), for the layouts Pillow cannot write (4:4:0,
 * 4:1:1).  Usage: mk_sampled_jpeg W H quality h v restart_blocks in.rgb out.jpg */
#include <stdio.h>
#include <stdlib.h>

#include <jpeglib.h>

int main(int argc, char** argv)
{
    if (argc != 9) return 2;
    const int w = atoi(argv[1]), h = atoi(argv[2]), q = atoi(argv[3]), hs = atoi(argv[4]), vs = atoi(argv[5]),
              rb = atoi(argv[6]);
    FILE* fi = fopen(argv[7], "rb");
    FILE* fo = fopen(argv[8], "wb");
    if (!fi || !fo) return 3;
    unsigned char* px = malloc((size_t)w * h * 3);
    if (fread(px, 1, (size_t)w * h * 3, fi) != (size_t)w * h * 3) return 4;
    struct jpeg_compress_struct c;
    struct jpeg_error_mgr e;
    c.err = jpeg_std_error(&e);
    jpeg_create_compress(&c);
    jpeg_stdio_dest(&c, fo);
    c.image_width = w;
    c.image_height = h;
    c.input_components = 3;
    c.in_color_space = JCS_RGB;
    jpeg_set_defaults(&c);
    jpeg_set_quality(&c, q, TRUE);
    c.comp_info[0].h_samp_factor = hs;
    c.comp_info[0].v_samp_factor = vs;
    for (int k = 1; k < 3; k++) c.comp_info[k].h_samp_factor = c.comp_info[k].v_samp_factor = 1;
    c.restart_interval = rb;
    c.optimize_coding = FALSE;
    jpeg_start_compress(&c, TRUE);
    while (c.next_scanline < c.image_height) {
        JSAMPROW row = px + (size_t)c.next_scanline * w * 3;
        jpeg_write_scanlines(&c, &row, 1);
    }
    jpeg_finish_compress(&c);
    jpeg_destroy_compress(&c);
    fclose(fo);
    fclose(fi);
    free(px);
    return 0;
}
