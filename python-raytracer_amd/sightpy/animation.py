"""Frame loops over `Scene.render` (reference `sightpy/animation.py:6-54`).

Same frames, files and order as the reference.  Two things keep a frame sequence on the GPU's
pace: the scene's device tables persist across frames (the texel pool stays
in HBM while the scene uses the same images, srt_scene_desc.texel_key; only the small collider /
material tables are re-sent after `update_scene`), and encoding and writing frame i overlaps the
rendering of frame i+1 (a background writer thread; every file is complete when the function
returns).
"""
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

__all__ = ["create_animation", "create_animation_using_opencv"]


def create_animation(scene, samples_per_pixel, fps, start_time, final_time, update_scene, name):
    number_of_frames = int(fps * (final_time - start_time))
    dt = (final_time - start_time) / number_of_frames
    t = start_time
    Path("./frames").mkdir(exist_ok=True)
    with ThreadPoolExecutor(max_workers=2) as writer:
        pending = []
        for i in range(number_of_frames):
            update_scene(scene, t)
            img = scene.render(samples_per_pixel)
            t += dt
            pending.append(writer.submit(img.save, "frames/" + name + "_" + str(i) + ".png"))
        for f in pending:
            f.result()  # re-raise write errors


def create_animation_using_opencv(scene, samples_per_pixel, fps, start_time, final_time, update_scene, name):
    import cv2

    number_of_frames = int(fps * (final_time - start_time))
    dt = (final_time - start_time) / number_of_frames
    t = start_time
    dims = (scene.camera.screen_width, scene.camera.screen_height)
    video = cv2.VideoWriter(name, cv2.VideoWriter_fourcc("M", "J", "P", "G"), fps, dims)
    # frames must reach the writer in order: one writer thread, frames queued in order
    with ThreadPoolExecutor(max_workers=1) as writer:
        pending = []
        for i in range(number_of_frames):
            update_scene(scene, t)
            frame = scene.render(samples_per_pixel)
            pending.append(writer.submit(lambda f: video.write(cv2.cvtColor(np.array(f), cv2.COLOR_RGB2BGR)), frame))
            t += dt
        for f in pending:
            f.result()
    video.release()
