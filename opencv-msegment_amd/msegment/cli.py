"""Console entry point mirroring the reference CLI.

Reference: src/main/java/ru/shayhulud/opencvcmsegment/App.java:14-31
  * exactly three arguments ``picturePath outMainFolder pictureName`` ("error parsing args"
    otherwise), each echoed as ``arg %d: %s``;
  * ``colorAutoMarkerWatershed(args...)`` then ``shapeAutoMarkerWatershed(args...)``
    (PictureService.java:290-299, :384-393), which read ``picturePath/pictureName``
    (readPicture, :117-159) and run the pipelines with no options.

The reference's console path keeps every step image in memory and never writes it (readPicture's
output folder is a TODO, :129-131; only the GUI's saveResultsToFS, :194-233, writes).  ``--save``
writes both methods' ``result`` and ``bw_result`` the way saveResultsToFS would, into
``outMainFolder/<name>_output/``, named by OutFileNameGenerator.generatePng
(common/util/OutFileNameGenerator.java:14-16): ``<METHOD>_<name>_<step %05d>_<stepName>.png``.
The step numbers are the ones the reference gives with NO_SAVE_STEPS (result 1, bw_result 2).
The colour method's contour numbering is unpinned against a real OpenCV build.

    python -m msegment.cli <picturePath> <outMainFolder> <pictureName> [--save] [--seed S]
"""
import os
import sys


def generate_png(filename, step, step_name):
    """OutFileNameGenerator.generatePng (OutFileNameGenerator.java:14-16)."""
    return "%s_%05d_%s.png" % (filename, step, step_name)


def image_file_name(picture_name):
    """ImageInfo.imageFileName: the picture name up to its first dot (PictureService.java:154)."""
    return picture_name.split(".")[0]


def read_picture(picture_path, picture_name):
    """readPicture (PictureService.java:117-159): the file decoded to a BGR uint8 array
    (Imgcodecs.imread's default IMREAD_COLOR); IOError when it cannot be decoded."""
    import numpy as np
    from PIL import Image

    full = os.path.join(picture_path, picture_name)
    try:
        with Image.open(full) as im:
            rgb = np.asarray(im.convert("RGB"), dtype=np.uint8)
    except (OSError, ValueError) as e:
        raise IOError("cannot read %s: %s" % (full, e)) from e
    return np.ascontiguousarray(rgb[:, :, ::-1])


def write_png(path, arr):
    import numpy as np
    from PIL import Image

    a = np.asarray(arr, dtype=np.uint8)
    Image.fromarray(a if a.ndim == 2 else np.ascontiguousarray(a[:, :, ::-1])).save(path)


def run(argv, out=sys.stdout, service=None):
    save = "--save" in argv
    seed = None
    args = []
    it = iter(argv)
    for a in it:
        if a == "--save":
            continue
        if a == "--seed":
            seed = int(next(it))
            continue
        args.append(a)
    if len(args) != 3:
        print("error parsing args", file=out)
        return 1
    for i, a in enumerate(args):
        print("arg %d: %s" % (i, a), file=out)
    picture_path, out_main_folder, picture_name = args
    try:
        src = read_picture(picture_path, picture_name)
    except IOError as e:
        print("There is an error with file stream processing: %s" % e, file=out)
        return 2
    if service is None:
        from .picture_service import PictureService

        service = PictureService(seed=seed)
    name = image_file_name(picture_name)
    # App.java:28: colorAutoMarkerWatershed(args...) -- contour numbering unpinned
    cres = service.color_auto_marker_watershed(src)
    print("colorAutoMarkerWatershed: %dx%d, depth %d" % (src.shape[0], src.shape[1], cres.depth), file=out)
    if save:
        odir = os.path.join(out_main_folder, name + "_output")
        os.makedirs(odir, exist_ok=True)
        for step, step_name, img in ((1, "result", cres.dst), (2, "bw_result", cres.bw)):
            path = os.path.join(odir, generate_png("COLOR_METHOD_" + name, step, step_name))
            write_png(path, img)
            print("wrote image %s" % path, file=out)
    # App.java:29: shapeAutoMarkerWatershed(args...)
    res = service.shape_auto_marker_watershed(src)
    if res is None:
        print("contours is empty", file=out)  # PictureService.java:451-453
        return 0
    print("shapeAutoMarkerWatershed: %dx%d, depth %d" % (src.shape[0], src.shape[1], res.depth), file=out)
    if save:
        odir = os.path.join(out_main_folder, name + "_output")
        os.makedirs(odir, exist_ok=True)
        for step, step_name, img in ((1, "result", res.dst), (2, "bw_result", res.bw)):
            path = os.path.join(odir, generate_png("SHAPE_METHOD_" + name, step, step_name))
            write_png(path, img)
            print("wrote image %s" % path, file=out)
    return 0


def main():
    sys.exit(run(sys.argv[1:]))


if __name__ == "__main__":
    main()
